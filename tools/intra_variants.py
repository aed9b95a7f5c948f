#!/usr/bin/env python3
"""Timing of the lowres intra estimate (x264hip_*_lowres_intra_cost) at 1080p over
F lowres frames: SATD with all 10 modes / DC-H-V only, SAD; after a clock-settling
warmup.  VALU lane-ops per block are read from the kernel's ISA (tools/README)."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package(); x.init(0)
from x264hip import synth
res = {}
for F in (16, 64):
    for bd in (8, 10):
        W, H = 1920, 1088
        mbw, mbh = W // 16, H // 16
        base, stride, origin = synth.make_sequence(17, W, H, bd)
        planes = np.concatenate([base] * ((F + 16) // 17))[:F]
        dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
        outs, ls = x.frame_init_lowres(dev, origin, stride, W, H)
        low = outs[0]
        for name, satd, allm, var, rows in (("satd_all", True, True, "0", True), ("satd_all_v1", True, True, "1", True),
                                            ("satd_all_norows", True, True, "0", False),
                                            ("satd_dhv", True, False, "0", True), ("sad_all", False, True, "0", True)):
            sys.modules["x264hip"].set_variant("X264HIP_LOWRES_INTRA_VARIANT", var)
            o = x.lowres_intra_cost(low, ls, mbw, mbh, satd, allm, 1, with_rows=rows)
            run = lambda: x.lowres_intra_cost(low, ls, mbw, mbh, satd, allm, 1, outs=o)  # noqa
            for _ in range(150):
                run()
            ts = []
            for _ in range(5):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    run()
                e.record(); torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 10)
            ms = float(np.median(ts))
            res[f"F{F}_bd{bd}_{name}"] = {"ms": ms, "mbs_per_s": F * mbw * mbh / ms * 1e3}
print(json.dumps(res, indent=1))
