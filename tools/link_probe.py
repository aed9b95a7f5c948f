#!/usr/bin/env python3
"""Host-link ceiling probe: pinned host -> HBM rates of
* one 256 MB buffer and 8.68 MB frames (one 2160p padded luma plane, configs[3]),
* the runtime's copy engine (hipMemcpyAsync via torch copy_) and x264hip_upload
  (a kernel reading the pinned pages),
* on 1, 2 and 4 copy streams (each frame split into equal slices, one per stream).

Prints one JSON object (GB/s = 1e9 bytes/s).  Usage: python3 tools/link_probe.py [out.json]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def rate(fn, nbytes, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return nbytes * reps / dt / 1e9, dt / reps * 1e3


def main():
    x = load_package()
    x.init(0)
    out = {"device": torch.cuda.get_device_name(0)}
    for label, nbytes, reps in (("256MB", 256 << 20, 20), ("frame_8.68MB", 3904 * 2224, 200)):
        nbytes = (nbytes + 4095) & ~4095
        host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        host.random_(0, 255)
        dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        for nstreams in (1, 2, 4):
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            sl = nbytes // nstreams
            cur = torch.cuda.current_stream()

            def copy_sdma():
                for i, s in enumerate(streams):
                    s.wait_stream(cur)
                    with torch.cuda.stream(s):
                        dev[i * sl:(i + 1) * sl].copy_(host[i * sl:(i + 1) * sl], non_blocking=True)
                for s in streams:
                    cur.wait_stream(s)

            def copy_kernel():
                for i, s in enumerate(streams):
                    s.wait_stream(cur)
                    with torch.cuda.stream(s):
                        x.upload(dev[i * sl:(i + 1) * sl], host[i * sl:(i + 1) * sl])
                for s in streams:
                    cur.wait_stream(s)

            for how, fn in (("sdma", copy_sdma), ("kernel", copy_kernel)):
                gbs, ms = rate(fn, nbytes, reps)
                out[f"{label}_{how}_{nstreams}s_GBps"] = round(gbs, 2)
                out[f"{label}_{how}_{nstreams}s_ms"] = round(ms, 4)
            if not torch.equal(dev.cpu(), host):
                raise SystemExit("link_probe: copy mismatch")
        # device -> device copy of the same size, for scale
        d2 = torch.empty_like(dev)
        gbs, ms = rate(lambda: d2.copy_(dev), 2 * nbytes, reps)
        out[f"{label}_d2d_GBps_rw"] = round(gbs, 1)
        del host, dev, d2
    keys = [k for k in out if k.startswith("frame_8.68MB") and k.endswith("GBps")]
    out["frame_best"] = max(keys, key=lambda k: out[k])
    out["frame_best_GBps"] = out[out["frame_best"]]
    keys = [k for k in out if k.startswith("256MB") and k.endswith("GBps") and "d2d" not in k]
    out["large_best"] = max(keys, key=lambda k: out[k])
    out["large_best_GBps"] = out[out["large_best"]]
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
