#!/usr/bin/env python3
"""A/B of the lookahead wavefront's band height (X264HIP_LOOKAHEAD_BAND: block rows per
single-wave workgroup) on the bench's lookahead legs: the P search over 15 1080p lowres
pairs and the B costs over 14 triplets; every band height must give the default's
results bit for bit."""
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

F, W, H = 16, 1920, 1088
mbw, mbh = W // 16, H // 16
planes, stride, origin = synth.make_sequence(F, W, H, 8)
dev = torch.from_numpy(planes).cuda()
lw, lh = W, H
louts, _ = x.frame_init_lowres(dev, origin, stride, lw, lh)
ls_ = x.plane_stride(lw // 2)
iouts = x.lowres_intra_cost(louts[0], ls_, mbw, mbh, True, True, 1)
span = 8 * 512
ii = np.arange(span + 1, dtype=np.float32)
logs = np.where(ii == 0, np.float32(0.718), np.log2(ii + np.float32(1)) * np.float32(2) + np.float32(1.718))
half = np.minimum((logs.astype(np.float32) + np.float32(0.5)).astype(np.int64), 65535).astype(np.uint16)
cm = torch.from_numpy(np.concatenate([half[:0:-1], half]).view(np.int16)).cuda()
lref = [p[:-1] for p in louts]
lint = iouts[0][1:]
p1m = x.lowres_inter_cost(louts[0][2:], [p[:-2] for p in louts], ls_, mbw, mbh, iouts[0][2:], (cm, span))[0]
nt = F - 2


def run_p(outs=None):
    return x.lowres_inter_cost(louts[0][1:], lref, ls_, mbw, mbh, lint, (cm, span), outs=outs)


def run_b(outs=None):
    bm = [torch.empty((nt, mbw * mbh, 2), dtype=torch.int16, device="cuda") for _ in range(2)]
    bk = [torch.empty((nt, mbw * mbh), dtype=torch.int32, device="cuda") for _ in range(2)]
    o = x.lowres_bidir_cost(louts[0][1:-1], [p[:-2] for p in louts], [p[2:] for p in louts], ls_, mbw, mbh,
                            (cm, span), 3, bm[0], bk[0], bm[1], bk[1], p1_mvs=p1m, outs=outs)
    return list(o) + bm + bk


def flat(o):
    return [t.clone() for t in (o if isinstance(o, (list, tuple)) else [o]) if torch.is_tensor(t)]


bands = [16, 8, 4, 2]
ref = {}
res = {}
for b in bands:
    x.set_variant("X264HIP_LOOKAHEAD_BAND", b)
    po = flat(run_p())
    bo = flat(run_b())
    torch.cuda.synchronize()
    if not ref:
        ref = {"p": po, "b": bo}
    else:
        assert all(torch.equal(a, c) for a, c in zip(ref["p"], po)), ("P differs", b)
        assert all(torch.equal(a, c) for a, c in zip(ref["b"], bo)), ("B differs", b)
for _ in range(30):
    run_p()
times = {b: {"p": [], "b": []} for b in bands}
for rnd in range(3):
    for b in bands:
        x.set_variant("X264HIP_LOOKAHEAD_BAND", b)
        for leg, fn in (("p", run_p), ("b", run_b)):
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[b][leg].append(s.elapsed_time(e) / 5)
for b in bands:
    res["band%d" % b] = {k: round(float(np.median(v)), 3) for k, v in times[b].items()}
print(json.dumps(res))
