"""A/B of the plane SSD kernels (bench.py's ssd leg: 16 1080p pairs per launch):
default plane_ssd2_kernel vs X264HIP_SSD_VARIANT=1, interleaved, 8 and 10 bit."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402


class A:
    steps, warmup, width, height = 200, 100, 1920, 1088


x = load_package()
x.init(0)
from x264hip import synth  # noqa: E402
F = 16
res = {}
for bd in (8, 10):
    planes, stride, origin = synth.make_sequence(F + 1, A.width, A.height, bd)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    for rnd in range(3):
        for v in (None, "1"):
            x.set_variant("X264HIP_SSD_VARIANT", v)
            r = bench.rates_ssd(x, A, 1, dev, origin, stride, F)
            res.setdefault(f"bd{bd}_{v or 'ssd2'}", []).append(round(r["ssd_plane_launch_ms"] * 1e3, 2))
print(json.dumps({k: {"us": v, "hbm_frac_best": round(F * 2 * A.width * A.height * (2 if "bd10" in k else 1)
                                                      / (min(v) * 1e-6) / bench.HBM_PEAK, 3)} for k, v in res.items()}))
