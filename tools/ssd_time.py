"""Time bench.py's plane-SSD leg alone (16 1080p pairs, graph-timed).  Usage: python tools/ssd_time.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402


class A:
    steps, warmup, width, height = 50, 100, 1920, 1080


x = load_package()
x.init(0)
from x264hip import synth  # noqa: E402
planes, stride, origin = synth.make_sequence(17, 1920, 1088, 8)
dev = torch.from_numpy(planes).cuda()
bench._SETTLE_S = 0.04
out = [bench.rates_ssd(x, A, 1, dev, origin, stride, 16) for _ in range(3)]
print(json.dumps(out))
