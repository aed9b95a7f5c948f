#!/usr/bin/env python3
"""A/B of the fused reconstruction kernels (X264HIP_RECON_VARIANT: default = block pairs for
transform 4 / packed transform 8 with sector-aligned waves, 2 = the same unshifted, 1 = lane
per block), 1080p, F frames, after a clock-settling warmup."""
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
    fsz = planes[0].size
    flat = [[16] * 64] * 8
    q4m, q4b, q8m, q8b = x.cqm_init(bd, flat)
    dq4, dq8 = x.cqm_dequant(flat)
    qp = 26 + 6 * (bd - 8)
    nmb = F * mbw * mbh
    qpm = torch.full((nmb,), qp, dtype=torch.int32, device="cuda")
    for t in (4, 8):
        mf, bias = (q4m[1, qp], q4b[1, qp]) if t == 4 else (q8m[1, qp], q8b[1, qp])
        dct, _ = x.mb_dct_quant(t, dev[1:], origin, stride, dev[:-1], origin + 2 * stride + 3, stride, mbw, mbh, F,
                                torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bias.copy()).cuda(),
                                fenc_frame_stride=fsz, pred_frame_stride=fsz)
        dmf = torch.from_numpy((dq4[1] if t == 4 else dq8[1]).copy()).cuda()
        outs = {v: torch.zeros_like(dev[:-1]) for v in (None, "2", "1")}
        run = lambda v: x.mb_dequant_idct_add(t, dct, mbw, mbh, F, dmf, qpm, dev[:-1], origin, stride, outs[v],  # noqa
                                              origin, stride, pred_frame_stride=fsz, recon_frame_stride=fsz)
        for v in outs:
            sys.modules["x264hip"].set_variant("X264HIP_RECON_VARIANT", v)
            run(v)
        torch.cuda.synchronize()
        assert torch.equal(outs[None], outs["1"]) and torch.equal(outs[None], outs["2"])
        sys.modules["x264hip"].set_variant("X264HIP_RECON_VARIANT", None)
        for _ in range(150):
            run(None)
        times = {v: [] for v in outs}
        for rnd in range(5):
            for v in outs:
                sys.modules["x264hip"].set_variant("X264HIP_RECON_VARIANT", v)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(3):
                    run(v)
                e.record(); torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / 3)
        cs = 2 if bd == 8 else 4
        ps = 1 if bd == 8 else 2
        alg = nmb * 256 * (cs + 2 * ps)
        for v in outs:
            ms = float(np.median(times[v]))
            res[f"bd{bd}_t{t}_v{v}"] = {"ms": ms, "hbm_frac": alg / ms / 1e6 / 8000}
sys.modules["x264hip"].set_variant("X264HIP_RECON_VARIANT", None)
out = json.dumps(res, indent=1)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
