#!/usr/bin/env python3
"""A/B of the full-search kernel variants in one process (interleaved rounds),
1080p, 16 frame pairs, range 16, 8 and 10 bit.  Each configuration is
(X264HIP_ME_VARIANT, X264HIP_ME_LEAD): variant 1 is the per-candidate reference
kernel, 3 / 5 the default 8 / 10-bit kernels, lead = rows of ref loads in flight
ahead of the row being summed.  Tables must agree bit for bit."""
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
    vs = [(1, 0)] + ([(3, k) for k in range(4)] + [(7, 1), (7, 2)] if bd == 8 else [(5, k) for k in range(3)])

    def setv(v):
        sys.modules["x264hip"].set_variant("X264HIP_ME_VARIANT", str(v[0]))
        sys.modules["x264hip"].set_variant("X264HIP_ME_LEAD", str(v[1]))

    def run(table=None):
        return x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, W // 16, H // 16, F, R,
                                table=table, fenc_frame_stride=fs, ref_frame_stride=fs)
    tab = {}
    for v in vs:
        setv(v)
        tab[v] = run()
    torch.cuda.synchronize()
    for v in vs:
        assert torch.equal(tab[vs[0]][..., :2 * R + 1], tab[v][..., :2 * R + 1]), ("variants disagree", v)
    setv(vs[-1])
    for _ in range(150):                              # clock ramp (tools/me_sustain.py)
        run(tab[vs[-1]])
    times = {v: [] for v in vs}
    for rnd in range(9):
        for v in vs:
            setv(v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                run(tab[v])
            e.record(); torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / 5)
    cands = F * (W // 16) * (H // 16) * 33 * 33
    for v in vs:
        ms = float(np.median(times[v]))
        res[f"bd{bd}_v{v[0]}_lead{v[1]}"] = {"ms": round(ms, 4), "Gcand_s": round(cands / ms / 1e6, 1),
                                             "T_absdiff_s": round(cands * 256 / ms / 1e9, 2)}
print(json.dumps(res, indent=1))
