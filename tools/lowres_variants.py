#!/usr/bin/env python3
"""A/B of the frame_init_lowres kernels (X264HIP_LOWRES_VARIANT: default = two output rows
per wave, 3 / 4 = one / four rows, 2 = one row per workgroup with a border wave, 1 = the
dword kernel) over F 1080p frames; every variant's planes must equal the default's."""
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
vs = [None, "3", "4", "2", "1"]
outs = {}
for v in vs:
    x.set_variant("X264HIP_LOWRES_VARIANT", v)
    outs[v], _ = x.frame_init_lowres(dev, origin, stride, W, H)
torch.cuda.synchronize()
for v in vs:
    assert all(torch.equal(a, b) for a, b in zip(outs[None], outs[v])), v
fb = planes[0].size
lbytes = fb + 4 * outs[None][0][0].numel()
for _ in range(200):
    x.set_variant("X264HIP_LOWRES_VARIANT", None)
    x.frame_init_lowres(dev, origin, stride, W, H, outs=outs[None])
times = {str(v): [] for v in vs}
for rnd in range(5):
    for v in vs:
        x.set_variant("X264HIP_LOWRES_VARIANT", v)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            x.frame_init_lowres(dev, origin, stride, W, H, outs=outs[v])
        e.record()
        torch.cuda.synchronize()
        times[str(v)].append(s.elapsed_time(e) / 10)
print(json.dumps({k: {"ms": round(float(np.median(t)), 4),
                      "hbm_frac": round(F * lbytes / (float(np.median(t)) * 1e-3) / 8e12, 3)} for k, t in times.items()}))
