#!/usr/bin/env python3
"""A/B of the 8-bit streaming frame kernels' launch forms, 16 and 64 1080p frames per launch,
interleaved rounds after a clock warmup; every form's outputs must equal the default's.
hpel_filter (X264HIP_HPEL_VARIANT 3, and 7 with default / forced nontemporal / plain stores) and
frame_init_lowres (the default two-row kernel with default / nontemporal / plain stores).  Usage: stream_var_ab.py [out.json]"""
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
planes, stride, origin = synth.make_sequence(64, W, H, 8)
full = torch.from_numpy(planes).cuda()
CONF = {"hpel": [{"X264HIP_HPEL_VARIANT": 3, "X264HIP_STREAM_NT": 0},
                 {"X264HIP_HPEL_VARIANT": 3},
                 {"X264HIP_HPEL_VARIANT": 7},
                 {"X264HIP_HPEL_VARIANT": 7, "X264HIP_STREAM_NT": 0},
                 {"X264HIP_HPEL_VARIANT": 7, "X264HIP_STREAM_XCD": 0}],
        "lowres": [{"X264HIP_LOWRES_VARIANT": -1},
                   {"X264HIP_LOWRES_VARIANT": -1, "X264HIP_STREAM_NT": 0}]}
NAMES = ("X264HIP_HPEL_VARIANT", "X264HIP_STREAM_XCD", "X264HIP_LOWRES_VARIANT", "X264HIP_STREAM_NT")


def setc(c):
    for n in NAMES:
        x.set_variant(n, c.get(n, None))


res = {}
for F in (16, 64):
    dev = full[:F]
    fb = dev[0].numel()
    hv = [[torch.zeros_like(dev) for _ in range(3)] for _ in CONF["hpel"]]
    lo = []
    for i, c in enumerate(CONF["hpel"]):
        setc(c)
        x.hpel_filter(dev, origin, stride, W, H, outs=hv[i])
    for i, c in enumerate(CONF["lowres"]):
        setc(c)
        lo.append(x.frame_init_lowres(dev, origin, stride, W, H)[0])
    torch.cuda.synchronize()
    for i in range(1, len(CONF["hpel"])):
        assert all(torch.equal(a, b) for a, b in zip(hv[0], hv[i])), ("hpel form changed the output", i)
    for i in range(1, len(CONF["lowres"])):
        assert all(torch.equal(a, b) for a, b in zip(lo[0], lo[i])), ("lowres form changed the output", i)
    lbytes = fb + 4 * lo[0][0][0].numel()
    legs = {"hpel": (lambda i: x.hpel_filter(dev, origin, stride, W, H, outs=hv[i]), 4 * fb),
            "lowres": (lambda i: x.frame_init_lowres(dev, origin, stride, W, H, outs=lo[i]), lbytes)}
    for name, (fn, per) in legs.items():
        setc(CONF[name][0])
        for _ in range(int(3200 / F)):
            fn(0)
        times = [[] for _ in CONF[name]]
        for rnd in range(8):
            for i, c in enumerate(CONF[name]):
                setc(c)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    fn(i)
                e.record()
                torch.cuda.synchronize()
                times[i].append(s.elapsed_time(e) / 10)
        for i, c in enumerate(CONF[name]):
            ms = float(np.median(times[i]))
            tag = "_".join("%s%s" % (k.split("_")[-1].lower()[:4], v) for k, v in c.items())
            res[f"{name}_F{F}_{tag}_ms"] = round(ms, 4)
            res[f"{name}_F{F}_{tag}_hbm_frac"] = round(F * per / (ms * 1e-3) / 8e12, 4)
    del hv, lo
setc({})
s = json.dumps(res, indent=1)
print(s)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(s + "\n")
