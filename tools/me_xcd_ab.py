#!/usr/bin/env python3
"""A/B of the headline full-search kernel (variant 7) with and without the XCD-contiguous
workgroup remap (X264HIP_ME_XCD), 1080p range 16, 16 and 64 frame pairs per launch,
interleaved rounds after a clock warmup.  Tables must agree bit for bit.
Usage: python3 tools/me_xcd_ab.py [out.json]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package  # noqa: E402

x = load_package()
x.init(0)
from x264hip import synth  # noqa: E402

W, H, R = 1920, 1088, 16
res = {}
planes, stride, origin = synth.make_sequence(65, W, H, 8)
dev = torch.from_numpy(planes).cuda()
fs = planes[0].size
for F in (16, 64):
    def run(table=None, F=F):
        return x.me_search_full(dev[1:F + 1], origin, stride, dev[:F], origin, stride, W // 16, H // 16, F, R,
                                table=table, fenc_frame_stride=fs, ref_frame_stride=fs)
    tabs = {}
    for v in (0, 1):
        x.set_variant("X264HIP_ME_XCD", v)
        tabs[v] = run()
    torch.cuda.synchronize()
    assert torch.equal(tabs[0][..., :2 * R + 1], tabs[1][..., :2 * R + 1]), "remap changed the table"
    for _ in range(int(2400 / F)):
        run(tabs[0])
    times = {0: [], 1: []}
    for rnd in range(10):
        for v in (0, 1):
            x.set_variant("X264HIP_ME_XCD", v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(int(80 / F)):
                run(tabs[v])
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / int(80 / F))
    for v in (0, 1):
        ms = float(np.median(times[v]))
        res[f"F{F}_xcd{v}_ms"] = round(ms, 4)
        res[f"F{F}_xcd{v}_frac"] = round(F * 8160 * 1089 * 256 / (ms * 1e-3) / 157.3e12, 4)
    del tabs
x.set_variant("X264HIP_ME_XCD", None)
s = json.dumps(res, indent=1)
print(s)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(s + "\n")
