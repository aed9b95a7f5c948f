#!/usr/bin/env python3
"""Where a lookahead search step's time goes: the P leg of bench.py (15 1080p lowres
pairs) timed with the search's options switched (DIA / HEX, subme 2 / 4, SATD on / off)."""
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

F, W, H = 16, 1920, 1088
mbw, mbh = W // 16, H // 16
planes, stride, origin = synth.make_sequence(F, W, H, 8)
dev = torch.from_numpy(planes).cuda()
louts, _ = x.frame_init_lowres(dev, origin, stride, W, H)
ls_ = x.plane_stride(W // 2)
iouts = x.lowres_intra_cost(louts[0], ls_, mbw, mbh, True, True, 1)
span = 8 * 512
ii = np.arange(span + 1, dtype=np.float32)
logs = np.where(ii == 0, np.float32(0.718), np.log2(ii + np.float32(1)) * np.float32(2) + np.float32(1.718))
half = np.minimum((logs.astype(np.float32) + np.float32(0.5)).astype(np.int64), 65535).astype(np.uint16)
cm = torch.from_numpy(np.concatenate([half[:0:-1], half]).view(np.int16)).cuda()
lref = [p[:-1] for p in louts]
lint = iouts[0][1:]
res = {}
for me, sub, satd in ((1, 4, True), (1, 4, False), (1, 2, True), (0, 4, True), (0, 2, False)):
    def run():
        x.lowres_inter_cost(louts[0][1:], lref, ls_, mbw, mbh, lint, (cm, span), me_method=me, subme=sub, satd=satd)
    for _ in range(10):
        run()
    ts = []
    for r in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            run()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 5)
    res["me%d_subme%d_satd%d" % (me, sub, satd)] = round(float(np.median(ts)), 3)
print(json.dumps(res))
