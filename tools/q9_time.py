"""Time the qpel 3x3 neighbourhood SATD 8x8 kernel (bench.py's configs[2] leg: every 8x8
block of 16 1080p frames around a half-pel centre) at 8 and 10 bit.
Usage: python tools/q9_time.py [library path, default the package's libx264hip.so]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

x = load_package()
if len(sys.argv) > 1:
    x.LIB_PATH = os.path.abspath(sys.argv[1])
x.init(0)
from x264hip import synth  # noqa: E402

F, W, H = 16, 1920, 1088
mbw, mbh = W // 16, H // 16
res = {"lib": os.path.relpath(x.LIB_PATH, ROOT)}
for bd in (8, 10):
    planes, stride, origin = synth.make_sequence(F + 1, W, H, bd)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fstride = planes[0].size
    hv = [torch.zeros_like(dev) for _ in range(3)]
    x.hpel_filter(dev[:-1], origin, stride, W, H, outs=[h[:-1] for h in hv])
    ys, xs = np.meshgrid(np.arange(mbh * 2), np.arange(mbw * 2), indexing="ij")
    bx, by = (xs.ravel() * 8).astype(np.int64), (ys.ravel() * 8).astype(np.int64)
    bfo, cxy = [], []
    for f in range(F):
        bfo.append((f + 1) * fstride + origin + by * stride + bx)
        cxy.append(np.stack([4 * bx + 12 + 2, 4 * by + 8 + 4 * f * (fstride // stride)], 1).astype(np.int32))
    bfo = torch.from_numpy(np.concatenate(bfo)).cuda()
    cxy = torch.from_numpy(np.concatenate(cxy)).cuda()
    sc9 = torch.empty((bfo.numel(), 9), dtype=torch.int32, device="cuda")
    flat = dev.view(-1)
    ref_planes = [dev.view(-1)] + [h.view(-1) for h in hv]

    def run():
        x.subpel_qpel9_batch(x.CMP_SATD, x.PIXEL_8x8, flat, stride, ref_planes, origin, stride, bfo, cxy, scores=sc9)
    for _ in range(400):
        run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            run()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 50)
    ms = float(np.median(ts))
    res[f"bd{bd}"] = {"ms": round(ms, 5), "frac": round(sc9.numel() * 636 / (ms * 1e-3) / 78.64e12, 4),
                      "checksum": int(sc9.sum().item())}
print(json.dumps(res))
