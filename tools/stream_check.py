#!/usr/bin/env python3
"""bench.py's rates_2160p in isolation (20 and 100 frames), to compare its streaming number
with tools/stream_probe.py's on the same box."""
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

x = bench.load_package()
torch.cuda.set_device(0)
x.init(0)
out = {}
for steps in (20, 100):
    a = types.SimpleNamespace(range=16, steps=steps, warmup=5)
    r = bench.rates_2160p(x, a, 1)
    out[steps] = {k: round(v, 4) if isinstance(v, float) else v for k, v in r.items() if "ms" in k}
bench._SETTLE_S = 0.04
a = types.SimpleNamespace(range=16, steps=20, warmup=5)
r = bench.rates_2160p(x, a, 1)
out["settle"] = {k: round(v, 4) if isinstance(v, float) else v for k, v in r.items() if "ms" in k}
print(json.dumps(out, indent=1))
