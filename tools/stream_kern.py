#!/usr/bin/env python3
"""Launch the 8-bit streaming frame kernels at the bench's 64-frame shape a fixed number of
times (for rocprofv3 counter passes): hpel_filter, frame_init_lowres."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import load_package
x = load_package(); x.init(0)
from x264hip import synth
W, H, F = 1920, 1088, 64
planes, stride, origin = synth.make_sequence(F, W, H, 8)
dev = torch.from_numpy(planes).cuda()
hv = [torch.empty_like(dev) for _ in range(3)]
lo = x.frame_init_lowres(dev, origin, stride, W, H)[0]
for _ in range(int(os.environ.get("REPS", "30"))):
    x.hpel_filter(dev, origin, stride, W, H, outs=hv)
    x.frame_init_lowres(dev, origin, stride, W, H, outs=lo)
torch.cuda.synchronize()
print("ok")
