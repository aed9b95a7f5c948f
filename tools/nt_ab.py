#!/usr/bin/env python3
"""A/B of nontemporal stores (X264HIP_STREAM_NT 0 / 1 / default) in the streaming frame
kernels at the bench's shapes: fused DCT+quant 4x4 / 8x8, hpel_filter and frame_init_lowres
over F (16 and 64) 1080p frames per launch, interleaved rounds after a clock warmup; every
setting's outputs must equal the plain-store ones.  Usage: nt_ab.py [out.json]"""
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

W, H = 1920, 1088
mbw, mbh = W // 16, H // 16
planes, stride, origin = synth.make_sequence(65, W, H, 8)
full = torch.from_numpy(planes).cuda()
fb = full[0].numel()
q4m, q4b, q8m, q8b = x.cqm_init(8, [[16] * 64] * 8)
mf4, bs4 = torch.from_numpy(q4m[1, 26].copy()).cuda(), torch.from_numpy(q4b[1, 26].copy()).cuda()
mf8, bs8 = torch.from_numpy(q8m[1, 26].copy()).cuda(), torch.from_numpy(q8b[1, 26].copy()).cuda()
SETS = (0, 1, None)
res = {}
for F in (16, 64):
    fenc, pred = full[1:F + 1], full[:F]
    nmb = F * mbw * mbh
    outs = {}
    legs = {}
    for s in SETS:
        dct = torch.empty((nmb, 256), dtype=torch.int16, device="cuda")
        nz = torch.empty(nmb, dtype=torch.int32, device="cuda")
        dct8 = torch.empty_like(dct)
        nz8 = torch.empty_like(nz)
        hv = [torch.zeros_like(pred) for _ in range(3)]
        lo = x.frame_init_lowres(pred, origin, stride, W, H)[0]
        outs[s] = (dct, nz, dct8, nz8, hv, lo)
    fs = fb

    def mk(s):
        dct, nz, dct8, nz8, hv, lo = outs[s]
        return {
            "dct4": (lambda: x.mb_dct_quant(4, fenc, origin, stride, pred, origin, stride, mbw, mbh, F, mf4, bs4,
                                            dct=dct, nz=nz, fenc_frame_stride=fs, pred_frame_stride=fs),
                     nmb * 16 * 64),
            "dct8": (lambda: x.mb_dct_quant(8, fenc, origin, stride, pred, origin, stride, mbw, mbh, F, mf8, bs8,
                                            dct=dct8, nz=nz8, fenc_frame_stride=fs, pred_frame_stride=fs),
                     nmb * 4 * 256),
            "hpel": (lambda: x.hpel_filter(pred, origin, stride, W, H, outs=hv), F * 4 * fb),
            "lowres": (lambda: x.frame_init_lowres(pred, origin, stride, W, H, outs=lo),
                       F * (fb + 4 * lo[0][0].numel())),
        }
    fns = {s: mk(s) for s in SETS}
    for s in SETS:
        x.set_variant("X264HIP_STREAM_NT", s)
        for name, (fn, _) in fns[s].items():
            fn()
    torch.cuda.synchronize()
    for s in SETS[1:]:
        a, b = outs[0], outs[s]
        for i in range(4):
            assert torch.equal(a[i], b[i]), ("NT changed an output", s, i)
        assert all(torch.equal(p, q) for p, q in zip(a[4], b[4])), ("NT changed hpel", s)
        assert all(torch.equal(p, q) for p, q in zip(a[5], b[5])), ("NT changed lowres", s)
    for name in fns[0]:
        x.set_variant("X264HIP_STREAM_NT", 0)
        for _ in range(int(3200 / F)):
            fns[0][name][0]()
        times = {s: [] for s in SETS}
        for rnd in range(8):
            for s in SETS:
                x.set_variant("X264HIP_STREAM_NT", s)
                fn = fns[s][name][0]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[s].append(e0.elapsed_time(e1) / 10)
        for s in SETS:
            ms = float(np.median(times[s]))
            tag = "default" if s is None else "nt%d" % s
            res[f"{name}_F{F}_{tag}_ms"] = round(ms, 4)
            res[f"{name}_F{F}_{tag}_hbm_frac"] = round(fns[s][name][1] / (ms * 1e-3) / 8e12, 4)
    del outs, fns
x.set_variant("X264HIP_STREAM_NT", None)
out = json.dumps(res, indent=1)
print(out)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(out + "\n")
