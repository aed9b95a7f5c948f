#!/usr/bin/env python3
"""A/B of the full-search kernel variants in one process (interleaved rounds),
1080p, 16 frame pairs, range 16, 8 and 10 bit."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package(); x.init(0)
from x264hip import synth
res = {}
for bd in (8, 10):
    F, W, H, R = 16, 1920, 1088, 16
    planes, stride, origin = synth.make_sequence(F + 1, W, H, bd)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    vs = (1, 2, 3) if bd == 8 else (1, 2, 5)
    tab = {}
    for v in vs:
        sys.modules["x264hip"].set_variant("X264HIP_ME_VARIANT", str(v))
        tab[v] = x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, W // 16, H // 16, F, R,
                                  fenc_frame_stride=fs, ref_frame_stride=fs)
    torch.cuda.synchronize()
    for v in vs:
        assert torch.equal(tab[1][..., :2 * R + 1], tab[v][..., :2 * R + 1]), ("variants disagree", v)
    def setv(v):
        sys.modules["x264hip"].set_variant("X264HIP_ME_VARIANT", str(v))
    setv(vs[2])
    for _ in range(150):                              # clock ramp (tools/me_sustain.py)
        x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, W // 16, H // 16, F, R,
                         table=tab[vs[2]], fenc_frame_stride=fs, ref_frame_stride=fs)
    times = {v: [] for v in vs}
    for rnd in range(5):
        for v in vs:
            setv(v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, W // 16, H // 16, F, R,
                                 table=tab[v], fenc_frame_stride=fs, ref_frame_stride=fs)
            e.record(); torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / 5)
    cands = F * (W // 16) * (H // 16) * 33 * 33
    for v in vs:
        ms = float(np.median(times[v]))
        res[f"bd{bd}_v{v}"] = {"ms": ms, "Gcand_s": cands / ms / 1e6, "T_absdiff_s": cands * 256 / ms / 1e9}
print(json.dumps(res, indent=1))
