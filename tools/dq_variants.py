#!/usr/bin/env python3
"""A/B of the fused DCT+quant kernels (X264HIP_DQ_VARIANT 1 = block-major, default =
strip, 6/7 = packed 8-bit transform 8) in one process; 1080p, F frame pairs (default 64: working set > 256 MiB MALL)."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package(); x.init(0)
from x264hip import synth
F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
res = {}
VS = ("1", "2", "3", "4", "5", "6", "7", "0")
for bd in (8, 10):
    W, H = 1920, 1088
    base, stride, origin = synth.make_sequence(17, W, H, bd)
    planes = np.concatenate([base] * ((F + 1 + 16) // 17))[:F + 1]
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fsz = planes[0].size
    q4m, q4b, q8m, q8b = x.cqm_init(bd, [[16] * 64] * 8)
    qp = 26 + 6 * (bd - 8)
    nmb = F * (W // 16) * (H // 16)
    for t in (4, 8):
        mf, bias = (q4m[1, qp], q4b[1, qp]) if t == 4 else (q8m[1, qp], q8b[1, qp])
        mf, bias = torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bias.copy()).cuda()
        outs = {}
        times = {}
        for v in VS:
            sys.modules["x264hip"].set_variant("X264HIP_DQ_VARIANT", v)
            outs[v] = x.mb_dct_quant(t, dev[1:], origin, stride, dev[:-1], origin + 2 * stride + 3, stride, W // 16,
                                     H // 16, F, mf, bias, fenc_frame_stride=fsz, pred_frame_stride=fsz)
            times[v] = []
        torch.cuda.synchronize()
        for _ in range(150):        # settle the clocks (tools/me_sustain.py)
            x.mb_dct_quant(t, dev[1:], origin, stride, dev[:-1], origin + 2 * stride + 3, stride, W // 16,
                           H // 16, F, mf, bias, dct=outs["1"][0], nz=outs["1"][1], fenc_frame_stride=fsz,
                           pred_frame_stride=fsz)
        for v in VS[1:]:
            assert torch.equal(outs["1"][0], outs[v][0]) and torch.equal(outs["1"][1], outs[v][1]), v
        for rnd in range(5):
            for v in VS:
                sys.modules["x264hip"].set_variant("X264HIP_DQ_VARIANT", v)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(3):
                    x.mb_dct_quant(t, dev[1:], origin, stride, dev[:-1], origin + 2 * stride + 3, stride, W // 16,
                                   H // 16, F, mf, bias, dct=outs[v][0], nz=outs[v][1], fenc_frame_stride=fsz,
                                   pred_frame_stride=fsz)
                e.record(); torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / 3)
        ps = 1 if bd == 8 else 2
        cs = 2 if bd == 8 else 4
        alg = nmb * 256 * (2 * ps + cs) + nmb * 4
        for v in VS:
            ms = float(np.median(times[v]))
            res[f"bd{bd}_t{t}_v{v}"] = {"ms": ms, "Gblocks_s": nmb * (16 if t == 4 else 4) / ms / 1e6,
                                       "GBps": alg / ms / 1e6, "hbm_frac": alg / ms / 1e6 / 8000}
print(json.dumps(res, indent=1))
