#!/usr/bin/env python3
"""Run bench.py side legs alone on the bench's 16-pair 1080p workload (for rocprofv3 trace /
PMC passes and A/Bs): leg_time.py LEG [steps] [pairs] with LEG one of esa (the ESA table and
fused legs), refine (refine_subpel with chroma ME on the quarter-pel sequence), full8 (the quadrant tables),
tesa, la (the lookahead's P and B searches), wp (the weight search), me10 (configs[4]'s 10-bit
full search, quadrant tables and 8x8 DCT+quant), esa8 (the sub-partition ESA decisions beside the
quadrant tables).  Prints the legs' JSON."""
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    leg = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    F = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    x = bench.load_package()
    x.init(0)
    from x264hip import synth
    a = types.SimpleNamespace(steps=steps, warmup=5, range=16, tframes=64, width=1920, height=1080)
    W, H = 1920, 1088
    mbw, mbh = W // 16, H // 16
    planes, stride, origin = synth.make_sequence(F + 1, W, H, 8)
    dev = torch.from_numpy(planes).cuda()
    fs = planes[0].size
    if leg == "esa":
        res = bench.rates_esa(x, a, 1, dev, origin, stride, fs, mbw, mbh, F)
    elif leg == "refine":
        res = bench.rates_refine(x, a, 1, mbw, mbh, F)
    elif leg == "full8":
        res = bench.rates_full8(x, a, 1, dev, origin, stride, fs, mbw, mbh, F)
    elif leg == "esa8":
        res = bench.rates_full8(x, a, 1, dev, origin, stride, fs, mbw, mbh, F)
        res.update(bench.rates_esa8(x, a, 1, dev, origin, stride, fs, mbw, mbh, F))
    elif leg == "tesa":
        res = bench.rates_tesa(x, a, 1, dev, origin, stride, fs, mbw, mbh, F)
    elif leg == "la":
        louts, _ = x.frame_init_lowres(dev[:-1], origin, stride, W, H)
        iouts = x.lowres_intra_cost(louts[0], x.plane_stride(W // 2), mbw, mbh, True, True, 1)
        res = bench.rates_lookahead(x, a, 1, louts, iouts, W, mbw, mbh, F)
    elif leg == "me10":
        res = bench.rates_10bit(x, a, 1, mbw, mbh, F)
    elif leg == "wp":
        res = bench.rates_weightp(x, a, 1, dev, origin, stride, mbw, mbh)
        res.update(bench.rates_ssim(x, a, 1, dev, origin, stride, mbw, mbh))
    else:
        raise SystemExit("unknown leg %s" % leg)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
