#!/usr/bin/env python3
"""Time the fused DCT+quant legs of bench.py alone (64 1080p pairs, the prediction a
buffer of its own) for a PMC / trace pass: dq_time.py [frames] [iterations] [variant]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


# A/B over (X264HIP_STREAM_NT, X264HIP_STREAM_XCD) pairs, "d" = the default: the default
# kernels (sector-shifted strips, nontemporal stores), plain stores (0/d) and the XCD order
# on (d/1); a fourth argument "default" times the default alone (PMC passes).  DQ_BD=10:
# 10-bit planes.  (Kernel variants that lost their A/Bs were removed in round 4; their
# history is in git)
VARIANTS = ("d/d", "0/d", "d/1")
ROUNDS = 5


def main():
    global VARIANTS, ROUNDS
    if len(sys.argv) > 3:
        VARIANTS, ROUNDS = ("d/d",), 1
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    x = load_package()
    x.init(0)
    from x264hip import synth
    bd = int(os.environ.get("DQ_BD", "8"))
    W, H = 1920, 1088
    mbw, mbh = W // 16, H // 16
    planes, stride, origin = synth.make_sequence(F + 1, W, H, bd)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    pred = dev[:-1].clone()
    fs = planes[0].size
    q4m, q4b, q8m, q8b = x.cqm_init(bd, [[16] * 64] * 8)
    qp = 26 + 6 * (bd - 8)
    nmb = F * mbw * mbh
    dct = torch.empty((nmb, 256), dtype=torch.int16 if bd == 8 else torch.int32, device="cuda")
    nz = torch.empty(nmb, dtype=torch.int32, device="cuda")
    res = {"bit_depth": bd}
    ps = 1 if bd == 8 else 2
    for t in (4, 8):
        mf, bs = (q4m[1, qp], q4b[1, qp]) if t == 4 else (q8m[1, qp], q8b[1, qp])
        mf, bs = torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bs.copy()).cuda()

        def step():
            x.mb_dct_quant(t, dev[1:], origin, stride, pred, origin, stride, mbw, mbh, F, mf, bs, dct=dct, nz=nz,
                           fenc_frame_stride=fs, pred_frame_stride=fs)
        for _ in range(100):
            step()
        blocks = nmb * (16 if t == 4 else 4)
        bpb = (64 if t == 4 else 256) * ps
        res["dct%d_algorithmic_bytes" % t] = blocks * bpb
        times = {v: [] for v in VARIANTS}
        for _ in range(ROUNDS):                      # interleaved rounds (the clock drifts)
            for v in VARIANTS:
                dv, xv = v.split("/")
                x.set_variant("X264HIP_STREAM_NT", None if dv == "d" else int(dv))
                x.set_variant("X264HIP_STREAM_XCD", None if xv == "d" else int(xv))
                step()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(n):
                    step()
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / n)
        x.set_variant("X264HIP_STREAM_XCD", None)
        x.set_variant("X264HIP_STREAM_NT", None)
        for v in VARIANTS:
            ms = sorted(times[v])[len(times[v]) // 2]
            tag = "" if v == "d/d" else "_" + v.replace("/", "_")
            res["dct%d%s_ms" % (t, tag)] = ms
            res["dct%d%s_hbm_frac" % (t, tag)] = blocks * bpb / (ms * 1e-3) / 8e12
    print(json.dumps(res))


if __name__ == "__main__":
    main()
