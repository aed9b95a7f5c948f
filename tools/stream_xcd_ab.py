#!/usr/bin/env python3
"""A/B of the XCD-contiguous block order (X264HIP_STREAM_XCD) for the 8-bit streaming
frame kernels hpel_filter and frame_init_lowres, 16 and 64 1080p frames per launch,
interleaved rounds after a clock warmup; outputs must agree bit for bit.
Usage: python3 tools/stream_xcd_ab.py [out.json]"""
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

W, H = 1920, 1088
planes, stride, origin = synth.make_sequence(64, W, H, 8)
full = torch.from_numpy(planes).cuda()
res = {}
for F in (16, 64):
    dev = full[:F]
    fb = dev[0].numel()
    hv = {v: [torch.zeros_like(dev) for _ in range(3)] for v in (0, 1)}
    lo = {}
    for v in (0, 1):
        x.set_variant("X264HIP_STREAM_XCD", v)
        x.hpel_filter(dev, origin, stride, W, H, outs=hv[v])
        lo[v], _ = x.frame_init_lowres(dev, origin, stride, W, H)
    torch.cuda.synchronize()
    for a, b in zip(hv[0] + list(lo[0]), hv[1] + list(lo[1])):
        assert torch.equal(a, b), "block order changed an output"
    lbytes = fb + 4 * lo[0][0][0].numel()
    legs = {"hpel": (lambda v: x.hpel_filter(dev, origin, stride, W, H, outs=hv[v]), 4 * fb),
            "lowres": (lambda v: x.frame_init_lowres(dev, origin, stride, W, H, outs=lo[v]), lbytes)}
    for name, (fn, per) in legs.items():
        for _ in range(int(3200 / F)):
            fn(0)
        times = {0: [], 1: []}
        for rnd in range(8):
            for v in (0, 1):
                x.set_variant("X264HIP_STREAM_XCD", v)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    fn(v)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / 10)
        for v in (0, 1):
            ms = float(np.median(times[v]))
            res[f"{name}_F{F}_xcd{v}_ms"] = round(ms, 4)
            res[f"{name}_F{F}_xcd{v}_hbm_frac"] = round(F * per / (ms * 1e-3) / 8e12, 4)
    del hv, lo
x.set_variant("X264HIP_STREAM_XCD", None)
s = json.dumps(res, indent=1)
print(s)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(s + "\n")
