#!/usr/bin/env python3
"""Regenerates tests/golden/intra8x8_golden.npz — TEST INFRASTRUCTURE.

Pins the oracle's closed-form 8x8 directional intra predictors (oracle.c
pred8x8_px: DDL, DDR, VR, HD, VL, HU) against the reference's own per-pixel
assignment lists in common/predict.c:741-883.  The reference's predict.c needs
the configure-generated config.h and cannot be compiled here, so this script
reads that file as text: every `SRC(x,y)=...= F2(...)` / `pack_pixel_*`
statement of the six functions is turned into a table "pixel (x,y) of mode m is
F1/F2 of these edge[] indices", and the tables are evaluated on random edges.
Only the resulting data (edges and predicted blocks) is committed; the tests
read the .npz and never the reference.

usage: python tests/golden/make_intra_golden.py   (needs /root/reference)
"""
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/common/predict.c"
MODES = ("ddl", "ddr", "vr", "hd", "vl", "hu")   # I_PRED_8x8_DDL .. I_PRED_8x8_HU = 3 .. 8


def edge_index(name):
    """edge[] slot of a neighbour name: l0..l7 -> 14..7, lt -> 15, t0..t15 -> 16..31"""
    if name == "lt":
        return 15
    if name[0] == "l":
        return 14 - int(name[1:])
    return 16 + int(name[1:])


def parse_term(term):
    """'F2(a,b,c)' / 'F1(a,b)' / 'l7' -> (kind, [edge indices])"""
    term = term.strip()
    m = re.fullmatch(r"(F[12])\((.*)\)", term)
    if m:
        return m.group(1), [edge_index(a.strip()) for a in m.group(2).split(",")]
    return "id", [edge_index(term)]


def mode_table(text, name):
    """{(x, y): (kind, indices)} for predict_8x8_<name>_c"""
    body = text[text.index(f"static void predict_8x8_{name}_c"):]
    body = body[:body.index("\n}\n")]
    table, pairs = {}, {}
    for line in (s.strip() for s in body.split("\n")):
        m = re.match(r"int (p\d+) = pack_pixel_1to2\((.*)\);", line)
        if m:
            args = re.findall(r"F[12]\([^)]*\)|\w+", m.group(2))
            pairs[m.group(1)] = [parse_term(a) for a in args]
        elif line.startswith("SRC_X4"):
            lhs, rhs = line.rstrip(";").split("= pack_pixel_2to4")
            a, b = (s.strip() for s in rhs.strip().strip("()").split(","))
            vals = pairs[a] + pairs[b]
            for xs, ys in re.findall(r"SRC_X4\((\d),(\d)\)", lhs):
                for k in range(4):
                    table[(int(xs) + k, int(ys))] = vals[k]
        elif line.startswith("SRC("):
            lhs, rhs = line.rstrip(";").rsplit("=", 1)
            for xs, ys in re.findall(r"SRC\((\d),(\d)\)", lhs):
                table[(int(xs), int(ys))] = parse_term(rhs)
    assert len(table) == 64, (name, len(table))
    return table


def evaluate(table, e):
    out = np.zeros((8, 8), np.int64)
    for (x, y), (kind, idx) in table.items():
        v = [int(e[i]) for i in idx]
        out[y, x] = (v[0] if kind == "id" else (v[0] + v[1] + 1) >> 1 if kind == "F1"
                     else (v[0] + 2 * v[1] + v[2] + 2) >> 2)
    return out


def main():
    text = open(REF).read()
    tables = [mode_table(text, m) for m in MODES]
    rs = np.random.default_rng(20261015)
    data = {}
    for bd in (8, 10):
        n = 64
        edges = rs.integers(0, 1 << bd, size=(n, 36)).astype(np.uint16)
        edges[0] = 0
        edges[1] = (1 << bd) - 1
        edges[2, ::2] = (1 << bd) - 1          # alternating extremes stress the rounding
        pred = np.zeros((n, len(MODES), 8, 8), np.uint16)
        for i in range(n):
            for k, t in enumerate(tables):
                pred[i, k] = evaluate(t, edges[i])
        data[f"edges_{bd}"] = edges
        data[f"pred_{bd}"] = pred
    np.savez_compressed(os.path.join(HERE, "intra8x8_golden.npz"), **data)
    print("wrote intra8x8_golden.npz")


if __name__ == "__main__":
    main()
