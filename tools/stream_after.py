#!/usr/bin/env python3
"""Which earlier bench leg slows the 2160p streaming leg?  Runs one leg of bench.py
(argv[1]: none | ssd | tesa | lowres | hpel | esa) on 16 1080p pairs, then rates_2160p."""
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

leg = sys.argv[1]
x = bench.load_package()
torch.cuda.set_device(0)
x.init(0)
from x264hip import synth  # noqa: E402
W, H, F = 1920, 1088, 16
planes, stride, origin = synth.make_sequence(F + 1, W, H, 8)
dev = torch.from_numpy(planes).cuda()
fs = planes[0].size
a = types.SimpleNamespace(range=16, steps=20, warmup=5, width=1920, height=1080, tframes=64)
bench._SETTLE_S = 0.04
if leg == "ssd":
    bench.rates_ssd(x, a, 1, dev, origin, stride, F)
elif leg == "tesa":
    bench.rates_tesa(x, a, 1, dev, origin, stride, fs, 120, 68, F)
elif leg == "esa":
    bench.rates_esa(x, a, 1, dev, origin, stride, fs, 120, 68, F)
elif leg == "hpel":
    hv = [torch.zeros_like(dev) for _ in range(3)]
    bench.timed(lambda: x.hpel_filter(dev[:-1], origin, stride, W, H, outs=[h[:-1] for h in hv]), 20, 5, 1,
                graph=True)
elif leg == "lowres":
    lo, _ = x.frame_init_lowres(dev, origin, stride, W, H)
    ic = x.lowres_intra_cost(lo[0], x.plane_stride(W // 2), 120, 68, True, True, 1)
    cm = torch.zeros(2 * 4096 + 1, dtype=torch.int16, device="cuda")
    x.lowres_inter_cost(lo[0][1:], [p[:-1] for p in lo], x.plane_stride(W // 2), 120, 68, ic[0][1:], (cm, 4096))
r = bench.rates_2160p(x, a, 1)
print(json.dumps({"leg": leg, "rounds": r["2160p_stream_rounds_ms"]}))
