#!/usr/bin/env python3
"""A/B of the 8-bit streaming half-pel kernel's strip height (X264HIP_HPEL_ROWS) over F
frames of 1080p, interleaved rounds after a clock-settling warmup; every configuration's
planes must equal the default's.  (Register-budget, non-temporal-store and packed-window
knobs were measured with this tool and dropped: none moved the kernel outside the noise.)"""
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

F = int(sys.argv[1]) if len(sys.argv) > 1 else 16
W, H = 1920, 1088
planes, stride, origin = synth.make_sequence(F, W, H, 8)
dev = torch.from_numpy(planes).cuda()
cfgs = [(r,) for r in (12, 6, 8, 16, 24)]
outs = {c: [torch.zeros_like(dev) for _ in range(3)] for c in cfgs}


def run(c):
    x.set_variant("X264HIP_HPEL_ROWS", c[0])
    x.hpel_filter(dev, origin, stride, W, H, outs=outs[c])


for c in cfgs:
    run(c)
torch.cuda.synchronize()
for c in cfgs:
    for a, b in zip(outs[cfgs[0]], outs[c]):
        assert torch.equal(a, b), ("configurations disagree", c)
for _ in range(200):
    run(cfgs[0])
times = {c: [] for c in cfgs}
for rnd in range(5):
    for c in cfgs:
        run(c)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run(c)
        e.record()
        torch.cuda.synchronize()
        times[c].append(s.elapsed_time(e) / 10)
alg = F * planes[0].size * 4
res = {}
for c in cfgs:
    ms = float(np.median(times[c]))
    res["rows%d" % c] = {"ms": round(ms, 4), "hbm_frac": round(alg / ms / 1e6 / 8000, 3)}
print(json.dumps(res, indent=1))
