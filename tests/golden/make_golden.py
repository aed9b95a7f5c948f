#!/usr/bin/env python3
"""Regenerates tests/golden/golden_{8,10}.npz — TEST INFRASTRUCTURE.

The reference publishes no golden vectors for this path and its C path is not
buildable here, so these fixtures freeze the outputs of the
oracle (oracle/oracle.c) on the reference's own checkasm inputs (glibc rand,
seed 12345, tools/checkasm.c) and on small synthetic frames.  Every value is
cross-checked against the independent numpy restatement before it is written.
Inputs are not stored; their SHA-256 is, so a drift of the input generators is
caught separately from a drift of the kernels.

usage: python tests/golden/make_golden.py
"""
import hashlib
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
ROOT = os.path.dirname(TESTS)
sys.path.insert(0, TESTS)

import checkasm_bufs as cb  # noqa: E402
import numpy_ref as nr  # noqa: E402
import oracle_lib as orc  # noqa: E402


def synth_module():
    spec = importlib.util.spec_from_file_location("synth", os.path.join(ROOT, "x264-i386pic_amd", "synth.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


OPS = ("sad", "ssd", "satd")
NPOPS = {"sad": nr.sad, "ssd": nr.ssd, "satd": nr.satd}
DCT_SHAPES = {"sub4x4_dct": (4, 4), "sub8x8_dct": (8, 8), "sub16x16_dct": (16, 16), "sub8x8_dct_dc": (8, 8),
              "sub8x16_dct_dc": (8, 16), "sub8x8_dct8": (8, 8), "sub16x16_dct8": (16, 16)}
NPDCT = {"sub4x4_dct": nr.sub4x4_dct, "sub8x8_dct": nr.sub8x8_dct, "sub16x16_dct": nr.sub16x16_dct,
         "sub8x8_dct_dc": nr.sub8x8_dct_dc, "sub8x16_dct_dc": nr.sub8x16_dct_dc, "sub8x8_dct8": nr.sub8x8_dct8,
         "sub16x16_dct8": nr.sub16x16_dct8}
QPS = (0, 6, 12, 20, 26, 33, 40, 47, 51)


def compute(bd):
    """All fixture arrays for one bit depth (inputs regenerated deterministically)."""
    out = {}
    b = cb.Bufs(bd)
    b.fill_pixel_overflow()
    out["in_sha_pixel"] = np.frombuffer(sha(b.pbuf1, b.pbuf3, b.pbuf4).encode(), np.uint8)
    pix = np.zeros((3, 8, 80), np.int32)
    for k, op in enumerate(OPS):
        for i, (w, h) in enumerate(nr.SIZES):
            for j in range(64):
                s1 = 32 if (j & 31) == 31 else 16
                v = orc.cmp(bd, op, i, b.pbuf1, 0, s1, b.pbuf1, b.pbuf2_off + j, 64)
                assert v == NPOPS[op](nr.block(b.pbuf1, 0, s1, w, h), nr.block(b.pbuf1, b.pbuf2_off + j, 64, w, h))
                pix[k, i, j] = v
            for t, j in enumerate(range(0, 0x1000, 256)):
                v = orc.cmp(bd, op, i, b.pbuf3, j, 16, b.pbuf4, j, 16)
                assert v == NPOPS[op](nr.block(b.pbuf3, j, 16, w, h), nr.block(b.pbuf4, j, 16, w, h))
                pix[k, i, 64 + t] = v
    out["pixel"] = pix
    x4 = np.zeros((2, 7, 64, 4), np.int32)
    for k, op in enumerate(("sad", "satd")):
        for i in range(7):
            for j in range(64):
                base = b.pbuf2_off + j
                x4[k, i, j] = orc.cmp_x(bd, op, 4, i, b.pbuf1, 0, b.pbuf1, [base, base + 6, base + 1, base + 10], 64)
    out["pixel_x4"] = x4

    b = cb.Bufs(bd)
    b.fill_dct_overflow()
    out["in_sha_dct"] = np.frombuffer(sha(b.pbuf1, b.pbuf3, b.pbuf4).encode(), np.uint8)
    for name, (w, h) in DCT_SHAPES.items():
        res = []
        for j in range(5):
            for (a, ao, d, do) in ((b.pbuf1, j * 64, b.pbuf1, b.pbuf2_off + j * 64),
                                   (b.pbuf3, 16 * j * 16, b.pbuf4, 16 * j * 32)):
                v = orc.sub_dct(bd, name, a, ao, d, do)
                want = NPDCT[name](nr.block(a, ao, 16, w, h) - nr.block(d, do, 32, w, h), bd)
                assert np.array_equal(v.astype(np.int64), want.ravel())
                res.append(v)
        out["dct_" + name] = np.stack(res)

    cb.srand(cb.SEED)
    cqm_all, quant_all = [], []
    for i_cqm in range(6):
        lists = cb.cqm_lists(i_cqm, bd)
        tabs = orc.cqm_init(bd, lists)
        for g, w in zip(tabs, nr.cqm_init(bd, lists)):
            assert np.array_equal(g, w)
        cqm_all.append(np.concatenate([t.ravel().astype(np.int64) for t in tabs]))
        q4m, q4b, q8m, q8b = tabs
        for qp in QPS:
            qp = min(qp + 6 * (bd - 8) if qp == 51 else qp, 51 + 6 * (bd - 8))
            c8 = cb.init_quant8(1, bd)
            c4 = cb.init_quant4(1, 16, bd)
            v8, n8 = orc.quant(bd, "quant_8x8", c8, q8m[1, qp], q8b[1, qp])
            v4, n4 = orc.quant(bd, "quant_4x4", c4, q4m[1, qp], q4b[1, qp])
            assert np.array_equal(v8, nr.quant(c8, q8m[1, qp], q8b[1, qp], bd)[0])
            assert np.array_equal(v4, nr.quant(c4, q4m[1, qp], q4b[1, qp], bd)[0])
            quant_all.append(np.concatenate([c8, v8.astype(np.int64), [n8], c4, v4.astype(np.int64), [n4]]))
    out["cqm"] = np.stack(cqm_all)
    out["quant"] = np.stack(quant_all)

    synth = synth_module()
    planes, stride, origin = synth.make_sequence(2, 64, 48, bd)
    out["in_sha_frames"] = np.frombuffer(sha(planes).encode(), np.uint8)
    out["me_full_r8"] = orc.me_search_full(bd, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride,
                                           4, 3, 8)
    q4m, q4b, q8m, q8b = orc.cqm_init(bd, [cb.FLAT16] * 8)
    qp = 26 + 6 * (bd - 8)
    d4, n4 = orc.mb_dct_quant(bd, 4, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, 4, 3,
                              q4m[1, qp], q4b[1, qp])
    d8, n8 = orc.mb_dct_quant(bd, 8, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, 4, 3,
                              q8m[1, qp], q8b[1, qp])
    out["mb_dct4_quant"], out["mb_dct4_nz"] = d4, n4
    out["mb_dct8_quant"], out["mb_dct8_nz"] = d8, n8
    return out


def main():
    for bd in (8, 10):
        arrays = compute(bd)
        path = os.path.join(HERE, f"golden_{bd}.npz")
        np.savez_compressed(path, **arrays)
        print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
