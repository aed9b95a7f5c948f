"""Time the TESA legs of bench.py alone (16 1080p pairs, me_range 16): the self-contained
kernel and the table-reading one.  Usage: python tools/tesa_time.py [centre_x centre_y]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402


class A:
    steps, warmup, range = 50, 100, 16


def main():
    x = load_package()
    if os.environ.get("TESA_LIB"):                   # an A/B build of the library
        x.LIB_PATH = os.path.abspath(os.environ["TESA_LIB"])
    x.init(0)
    from x264hip import synth
    W, H, F = 1920, 1088, 16
    mbw, mbh = W // 16, H // 16
    planes, stride, origin = synth.make_sequence(F + 1, W, H, 8)
    dev = torch.from_numpy(planes).cuda()
    if len(sys.argv) > 2:
        c = (int(sys.argv[1]), int(sys.argv[2]))
        orig = bench.tesa_params
        bench.tesa_params = lambda mbw, mbh, F, R: orig(mbw, mbh, F, R, centre=c)
    print(json.dumps(bench.rates_tesa(x, A, 1, dev, origin, stride, planes[0].size, mbw, mbh, F)))


if __name__ == "__main__":
    main()
