#!/usr/bin/env python3
"""Debug aid: where variant 7 of the half-pel filter differs from variant 3 (mismatch row /
column ranges per plane), for a few sizes and XCD orders."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package(); x.init(0)
from x264hip import synth
for (W, H) in ((176, 144), (1920, 1088)):
    planes, stride, origin = synth.make_sequence(2, W, H, 8)
    dev = torch.from_numpy(planes).cuda()
    res = {}
    for v, xcd in ((3, None), (7, None), (7, 0)):
        x.set_variant("X264HIP_HPEL_VARIANT", v)
        x.set_variant("X264HIP_STREAM_XCD", xcd)
        outs = [torch.full_like(dev, 7) for _ in range(3)]
        x.hpel_filter(dev, origin, stride, W, H, outs=outs)
        torch.cuda.synchronize()
        res[(v, xcd)] = [o.cpu().numpy() for o in outs]
    for key in ((7, None), (7, 0)):
        for p in range(3):
            a, b = res[(3, None)][p], res[key][p]
            d = np.argwhere(a != b)
            if len(d):
                f, r, c = d[:, 0], d[:, 1], d[:, 2]
                print(W, H, key, "plane", p, "n", len(d), "frames", sorted(set(f.tolist())), "rows", r.min(), r.max(),
                      "cols", c.min(), c.max(), "row hist", np.unique(r, return_counts=True)[0][:20],
                      "sample got/want", b[f[0], r[0], c[0]], a[f[0], r[0], c[0]], "untouched(7)", int((b == 7).sum()))
            else:
                print(W, H, key, "plane", p, "equal")
