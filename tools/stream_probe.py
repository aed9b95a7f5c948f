#!/usr/bin/env python3
"""configs[3] streaming-leg A/B: 2160p frames uploaded from pinned
host memory while the previous frame's full search (range 16) + fused 4x4 DCT+quant run.

Variants (each timed over --frames uploads after a warmup):
  upload how   : sdma (hipMemcpyAsync) | kernel (x264hip_upload) with a workgroup cap
  copy stream  : normal | high priority
  CU mask      : none | the copy stream on `reserve` CUs, the compute stream on the rest
                 (hipExtStreamCreateWithCUMask)
  batch        : frames per upload (1, or 2 adjacent frames in one transfer)

Prints one JSON object: per-variant ms per frame, plus upload-only and compute-only times.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def cu_mask_stream(L, bits, ncu):
    """A HIP stream restricted to the CUs whose bits are set (list of CU indices)."""
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    L.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_uint32)]
    L.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    rc = L.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), words)
    if rc:
        raise RuntimeError("hipExtStreamCreateWithCUMask: %d" % rc)
    return torch.cuda.ExternalStream(s.value)


def main():
    x = load_package()
    x.init(0)
    from x264hip import synth
    L = x.lib()
    nframes = int(os.environ.get("PROBE_FRAMES", "60"))
    W, H, R = 3840, 2160, 16
    mbw, mbh = W // 16, H // 16
    nf = 8
    planes, stride, origin = synth.make_sequence(nf + 1, W, H, 8)
    fsz = planes[0].size
    host = torch.from_numpy(planes).pin_memory()
    ring = torch.empty((4,) + planes.shape[1:], dtype=torch.uint8, device="cuda")
    table = torch.empty((1, mbh, mbw, 2 * R + 1, x.me_table_pitch(R)), dtype=torch.int16, device="cuda")
    flat = [16] * 64
    q4m, q4b, _, _ = x.cqm_init(8, [flat] * 8)
    mf4 = torch.from_numpy(q4m[1, 26].copy()).cuda()
    bs4 = torch.from_numpy(q4b[1, 26].copy()).cuda()
    dct = torch.empty((mbw * mbh, 256), dtype=torch.int16, device="cuda")
    nz = torch.empty(mbw * mbh, dtype=torch.int32, device="cuda")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    out = {"cus": ncu, "frame_bytes": int(fsz), "frames_timed": nframes}

    def work(cur, ref):
        x.me_search_full(cur, origin, stride, ref, origin, stride, mbw, mbh, 1, R, table=table,
                         fenc_frame_stride=0, ref_frame_stride=0)
        x.mb_dct_quant(4, cur, origin, stride, ref, origin, stride, mbw, mbh, 1, mf4, bs4, dct=dct, nz=nz,
                       fenc_frame_stride=0, pred_frame_stride=0)

    def run(label, how, wgs, copy, comp, nframes=nframes):
        x.set_variant("X264HIP_UPLOAD_WGS", wgs if wgs else None)
        done = [torch.cuda.Event() for _ in range(3)]
        ready = [torch.cuda.Event() for _ in range(3)]
        torch.cuda.synchronize()
        with torch.cuda.stream(comp):
            ring[0].copy_(host[0])
            ready[0].record(comp)
            for ev in done:
                ev.record(comp)
        torch.cuda.synchronize()

        def step(n):
            cur, ref = (n + 1) % 3, n % 3
            with torch.cuda.stream(copy):
                copy.wait_event(done[cur])
                if how == "sdma":
                    ring[cur].copy_(host[(n + 1) % (nf + 1)], non_blocking=True)
                else:
                    x.upload(ring[cur], host[(n + 1) % (nf + 1)])
                ready[cur].record(copy)
            with torch.cuda.stream(comp):
                comp.wait_event(ready[cur])
                comp.wait_event(ready[ref])
                work(ring[cur:cur + 1], ring[ref:ref + 1])
                done[ref].record(comp)
        for n in range(20):
            step(n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for n in range(20, 20 + nframes):
            step(n)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / nframes * 1e3
        out[label] = round(ms, 4)
        x.set_variant("X264HIP_UPLOAD_WGS", None)
        return ms

    def alone(label, fn, n=60):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        out[label] = round((time.perf_counter() - t0) / n * 1e3, 4)

    main_s = torch.cuda.current_stream()
    normal = torch.cuda.Stream()
    high = torch.cuda.Stream(priority=-1)
    alone("compute_only_ms", lambda: work(ring[1:2], ring[0:1]))
    alone("upload_sdma_only_ms", lambda: ring[1].copy_(host[1], non_blocking=True))
    alone("upload_kernel_only_ms", lambda: x.upload(ring[1], host[1]))
    for wgs in (16, 64):
        x.set_variant("X264HIP_UPLOAD_WGS", wgs)
        alone("upload_kernel_%dwg_only_ms" % wgs, lambda: x.upload(ring[1], host[1]))
        x.set_variant("X264HIP_UPLOAD_WGS", None)
    for how in ("sdma", "kernel"):
        run("%s_normal" % how, how, None, normal, main_s)
        run("%s_high" % how, how, None, high, main_s)
    for wgs in (16, 32, 64, 128):
        run("kernel_%dwg_normal" % wgs, "kernel", wgs, normal, main_s)
        run("kernel_%dwg_high" % wgs, "kernel", wgs, high, main_s)
    # CU masks: reserve the first k CU indices for the copy stream
    try:
        for k in (8, 16):
            cs = cu_mask_stream(L, range(k), ncu)
            ks = cu_mask_stream(L, range(k, ncu), ncu)
            alone("compute_only_masked%d_ms" % k, lambda: None)
            with torch.cuda.stream(ks):
                alone("compute_only_masked%d_ms" % k, lambda: work(ring[1:2], ring[0:1]))
            for wgs in (16, 64):
                run("kernel_%dwg_mask%d" % (wgs, k), "kernel", wgs, cs, ks)
            run("sdma_mask%d" % k, "sdma", None, cs, ks)
    except Exception as e:  # noqa: BLE001
        out["cu_mask_error"] = str(e)
    best = min((k for k in out if k.startswith(("sdma_", "kernel_")) and isinstance(out[k], float)),
               key=lambda k: out[k])
    out["best"] = best
    out["best_ms"] = out[best]
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
