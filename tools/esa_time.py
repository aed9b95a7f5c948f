"""Time the ESA legs of bench.py alone (16 1080p pairs, range 16): table path (headline
kernel + me_esa_argmin) and the fused search + decision."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402


class A:
    steps, warmup, range = 100, 150, 16


x = load_package()
x.init(0)
from x264hip import synth  # noqa: E402
W, H, F = 1920, 1088, 16
planes, stride, origin = synth.make_sequence(F + 1, W, H, 8)
dev = torch.from_numpy(planes).cuda()
print(json.dumps(bench.rates_esa(x, A, 1, dev, origin, stride, planes[0].size, W // 16, H // 16, F)))
