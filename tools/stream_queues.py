#!/usr/bin/env python3
"""Does the 2160p streaming pipeline serialise because its two streams share a hardware
queue?  Times bench.py's streaming leg after creating K other streams first (K = 0..5),
in one process each (argv[1] = K)."""
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

K = int(sys.argv[1])
x = bench.load_package()
torch.cuda.set_device(0)
x.init(0)
keep = [torch.cuda.Stream() for _ in range(K)]
a = types.SimpleNamespace(range=16, steps=20, warmup=5)
r = bench.rates_2160p(x, a, 1)
print(json.dumps({"K": K, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                  "rounds": r["2160p_stream_rounds_ms"]}))
