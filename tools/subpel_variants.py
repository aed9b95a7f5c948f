#!/usr/bin/env python3
"""A/B of the qpel candidate kernels (X264HIP_SUBPEL_VARIANT: 1 = lane per candidate with
dwordx2 + dword loads, 2 = row per lane, 3 = lane per candidate with unaligned multi-dword
row loads, 5 = single-dword row loads (default)) on bench.py's configs[2] list: 16 frames of 1080p, every 8x8 block, 9 qpel candidates
around a half-pel MV.  8 and 10 bit, SATD and SAD, interleaved rounds after a warmup."""
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
    mbw, mbh = W // 16, H // 16
    base, stride, origin = synth.make_sequence(17, W, H, bd)
    planes = np.concatenate([base] * ((F + 1 + 16) // 17))[:F + 1]
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fstride = planes[0].size
    hv = [torch.zeros_like(dev) for _ in range(3)]
    x.hpel_filter(dev[:-1], origin, stride, W, H, outs=[h[:-1] for h in hv])
    ys, xs = np.meshgrid(np.arange(mbh * 2), np.arange(mbw * 2), indexing="ij")
    bx, by = (xs.ravel() * 8).astype(np.int64), (ys.ravel() * 8).astype(np.int64)
    # list orders: "sweep" = per frame, per qpel offset, every block (one phase per
    # run of consecutive entries); "block" = per frame, per block, its 9 candidates
    # (refine_subpel's order)
    fo_s, q_s = [], []
    for f in range(F):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                fo_s.append((f + 1) * fstride + origin + by * stride + bx)
                q = np.stack([4 * bx + 12 + 2 + dx, 4 * by + 8 + dy], 1)
                q[:, 1] += 4 * f * (fstride // stride)
                q_s.append(q.astype(np.int32))
    nb = bx.size
    fo_s = np.concatenate(fo_s).reshape(F, 9, nb)
    q_s = np.concatenate(q_s).reshape(F, 9, nb, 2)
    orders = {"sweep": (fo_s.ravel(), q_s.reshape(-1, 2)),
              "block": (fo_s.transpose(0, 2, 1).ravel(), q_s.transpose(0, 2, 1, 3).reshape(-1, 2))}
    flat = dev.view(-1)
    ref_planes = [dev.view(-1)] + [h.view(-1) for h in hv]
    for (order, (fo_np, q_np)), op in [(o, op) for o in orders.items() for op in (2, 0)]:
        fo = torch.from_numpy(np.ascontiguousarray(fo_np)).cuda()
        qxy = torch.from_numpy(np.ascontiguousarray(q_np)).cuda()
        vs = ("1", "2", "3", "5") if op == 2 else ("1", "3", "5")
        sc = {v: torch.empty(fo.numel(), dtype=torch.int32, device="cuda") for v in vs}
        run = lambda v: x.subpel_cmp_batch(op, x.PIXEL_8x8, flat, stride, ref_planes, origin, stride, fo, qxy,  # noqa
                                           scores=sc[v])
        for v in vs:
            sys.modules["x264hip"].set_variant("X264HIP_SUBPEL_VARIANT", v)
            run(v)
        torch.cuda.synchronize()
        for v in vs:
            assert torch.equal(sc[vs[0]], sc[v]), ("variants disagree", bd, op, v)
        sys.modules["x264hip"].set_variant("X264HIP_SUBPEL_VARIANT", vs[-1])
        for _ in range(150):
            run(vs[-1])
        times = {v: [] for v in vs}
        for rnd in range(5):
            for v in vs:
                sys.modules["x264hip"].set_variant("X264HIP_SUBPEL_VARIANT", v)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    run(v)
                e.record(); torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / 5)
        for v in vs:
            ms = float(np.median(times[v]))
            res[f"bd{bd}_{order}_{'satd' if op == 2 else 'sad'}_v{v}"] = {"ms": round(ms, 4),
                                                                  "Gcand_s": round(fo.numel() / ms / 1e6, 1)}
    sys.modules["x264hip"].set_variant("X264HIP_SUBPEL_VARIANT", None)
    del dev, hv
print(json.dumps(res, indent=1))
