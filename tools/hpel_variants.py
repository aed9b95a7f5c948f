#!/usr/bin/env python3
"""A/B of the half-pel filter kernels (X264HIP_HPEL_VARIANT: 0 = fused LDS tiles,
1 = interior tiles + border expand, 2 = streaming lanes with scaled clamps, 3 = streaming
lanes with packed shift-saturate (8-bit default), 4 / 5 = 2 / 3 under a 4-waves-per-SIMD
register budget) on 16 frames
of 1080p, 8 and 10 bit, interleaved rounds after a clock-settling warmup."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package(); x.init(0)
from x264hip import synth
F = int(sys.argv[1]) if len(sys.argv) > 1 else 16
res = {}
for bd in (8, 10):
    W, H = 1920, 1088
    planes, stride, origin = synth.make_sequence(F, W, H, bd)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    vs = ("0", "1", "2", "3", "4", "5") if bd == 8 else ("0", "1")
    outs = {v: [torch.zeros_like(dev) for _ in range(3)] for v in vs}
    run = lambda v: x.hpel_filter(dev, origin, stride, W, H, outs=outs[v])  # noqa
    for v in vs:
        sys.modules["x264hip"].set_variant("X264HIP_HPEL_VARIANT", v)
        run(v)
    torch.cuda.synchronize()
    for v in vs:
        for a, b in zip(outs[vs[0]], outs[v]):
            assert torch.equal(a, b), ("variants disagree", bd, v)
    sys.modules["x264hip"].set_variant("X264HIP_HPEL_VARIANT", vs[-1])
    for _ in range(150):
        run(vs[-1])
    times = {v: [] for v in vs}
    for rnd in range(5):
        for v in vs:
            sys.modules["x264hip"].set_variant("X264HIP_HPEL_VARIANT", v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                run(v)
            e.record(); torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / 5)
    ps = 1 if bd == 8 else 2
    alg = F * planes[0].size * ps * 4          # one plane in, three out (padded planes)
    for v in vs:
        ms = float(np.median(times[v]))
        res[f"bd{bd}_v{v}"] = {"ms": round(ms, 4), "hbm_frac": round(alg / ms / 1e6 / 8000, 3)}
    sys.modules["x264hip"].set_variant("X264HIP_HPEL_VARIANT", None)
print(json.dumps(res, indent=1))
