#!/usr/bin/env python3
"""Practical HBM ceiling on the box: device-to-device copies (read + write) of several
sizes with torch, after a warmup long enough for the clocks to settle."""
import json, torch
res = {}
for mb in (32, 134, 512, 2048):
    n = mb * (1 << 20)
    a = torch.empty(n, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1)
    for _ in range(200 if mb < 512 else 40):
        b.copy_(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = 50 if mb < 512 else 10
    s.record()
    for _ in range(k):
        b.copy_(a)
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / k
    res[f"copy_{mb}MiB"] = {"ms": ms, "TBps_rw": 2 * n / ms / 1e9, "frac_of_8TBps": 2 * n / ms / 1e9 / 8.0}
    del a, b
print(json.dumps(res, indent=1))
