#!/usr/bin/env python3
"""A/B of the plane-SSD kernel's rows per wave (X264HIP_SSD_VARIANT 0 = 16, 1 = 8, 2 = 4) at 16
and 64 1080p pairs, graph-timed as bench.py's leg, interleaved rounds; outputs must agree."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402


class A:
    steps, warmup, width, height = 50, 100, 1920, 1080


x = load_package()
x.init(0)
from x264hip import synth  # noqa: E402
planes, stride, origin = synth.make_sequence(65, 1920, 1088, 8)
full = torch.from_numpy(planes).cuda()
bench._SETTLE_S = 0.04
res = {}
for F in (16, 64):
    dev = full[:F + 1]
    outs = []
    for v in (0, 1, 2):
        x.set_variant("X264HIP_SSD_VARIANT", v)
        o = torch.empty(F, dtype=torch.int64, device="cuda")
        x.ssd_plane_batch(dev[1:], origin, stride, dev[:-1].clone(), origin, stride, 1920, 1080, F, out=o)
        torch.cuda.synchronize()
        outs.append(o.cpu().numpy())
    assert all(np.array_equal(outs[0], o) for o in outs), "SSD variants disagree"
    t = {v: [] for v in (0, 1, 2)}
    for rnd in range(3):
        for v in (0, 1, 2):
            x.set_variant("X264HIP_SSD_VARIANT", v)
            t[v].append(bench.rates_ssd(x, A, 1, dev, origin, stride, F)["ssd_plane_launch_ms"])
    for v in (0, 1, 2):
        ms = float(np.median(t[v]))
        res["F%d_v%d_ms" % (F, v)] = round(ms, 4)
        res["F%d_v%d_hbm_frac" % (F, v)] = round(F * 2 * 1920 * 1080 / (ms * 1e-3) / 8e12, 4)
x.set_variant("X264HIP_SSD_VARIANT", None)
s = json.dumps(res, indent=1)
print(s)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(s + "\n")
