#!/usr/bin/env python3
"""Per-launch time of the 8-bit full search over a long back-to-back run
(clock / power behaviour under sustained load), 1080p, 16 pairs, range 16."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package(); x.init(0)
from x264hip import synth
F, W, H, R = 16, 1920, 1088, 16
bd = int(os.environ.get("BD", "8"))
planes, stride, origin = synth.make_sequence(F + 1, W, H, bd)
dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
fs = planes[0].size
tab = x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, W // 16, H // 16, F, R,
                       fenc_frame_stride=fs, ref_frame_stride=fs)
torch.cuda.synchronize()
out = {}
for n in (5, 200):
    torch.cuda._sleep(200_000_000)  # idle-ish gap (~0.1 s spin on one wave)
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    evs[0].record()
    for i in range(n):
        x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, W // 16, H // 16, F, R,
                         table=tab, fenc_frame_stride=fs, ref_frame_stride=fs)
        evs[i + 1].record()
    torch.cuda.synchronize()
    t = [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]
    out[n] = [round(v, 4) for v in t]
print(json.dumps(out))
