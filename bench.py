#!/usr/bin/env python3
"""bench.py — x264 motion-search / transform kernels on MI355X.

Metric (BASELINE.json): SAD+SATD candidate-MVs/sec + DCT+quant blocks/sec, 1080p.
Workload of the headline `value` (BASELINE.json configs[1]): 1080p synthetic luma,
full-search integer ME with range 16 (33x33 = 1089 16x16 SAD candidates per MB,
8160 MBs per frame), one step = one x264hip_8_me_search_full launch over
`--frames` (fenc, ref) pairs already resident in HBM.  value = candidates/s over
all ranks.  Side rates of configs[2] (SATD 8x8 candidates, fused 4x4 and 8x8
DCT+quant blocks) are measured in the same run and reported under "extra".

Multi-GPU: one process per GPU (torchrun), frames are sharded by rank (every
rank owns its own frame pairs: weak scaling, no data-path collective); the
barrier + max-over-ranks of the timed region use the default process group.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md): 256 CUs x 4 SIMD-32 at
# 2.4 GHz -> 78.6 T full-rate VALU lane-ops/s.  The byte-SAD instructions are not
# full rate (measured, profiles/r01_sad_peak.txt, r01_qsad_probe.txt): v_sad_u8
# (4 absdiffs) issues at 1/2 and v_qsad_pk_u16_u8 (16 absdiffs) at 1/8 of it, so
# both top out at 78.6e12 * 2 = 157.3 T byte-absdiffs/s — the SAD roofline.
VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9
SAD_PEAK_ABSDIFF = 2 * VALU_LANE_OPS          # 157.3 T absdiff/s
HBM_PEAK = 8.0e12


def workload_2160p(x, a, world, rank, pg_world, rank_dev):
    """configs[3] as its own bench line (--workload 2160p): one 2160p 4:2:0 frame per GPU per step,
    frame-per-GPU across the node (rank r encodes frames of its own shard; no collective on the
    data path).  The frames are synth.make_subpel_sequence's (quarter-pel motion (3.25, 2.5) px per
    frame, so the refine's diamonds move), held in pinned host memory as unpadded pictures, as
    x264_encoder_encode receives them.  A step = the new picture's luma and NV12 planes uploaded
    by x264hip_upload_plane (the PCIe read fused with x264_frame_expand_border) on the copy stream
    of a CU-partitioned stream pair (x264hip_stream_pair_create), overlapped with the previous
    step's kernels on the compute stream: its half-pel planes (it is the next step's reference),
    the exhaustive search of me.c:618-631 (range R around mv 0) against the previous frame with
    its decision, fused (x264hip_8_me_search_esa: no table in HBM), refine_subpel at
    subme 7 with chroma ME (x264's default preset on P slices: two hpel SAD diamonds, the SATD
    re-score with U / V, two qpel SATD diamonds, common/macroblock.c:507-509) from the decisions,
    and the fused 4x4 DCT + quant.  value = every rank's candidates (the table's (2R+1)^2 per MB
    + the refine's SAD / SATD calls, counted by the kernel) over the max-over-ranks wall of the
    timed steps, H2D included."""
    from x264hip import synth, dist as xd
    W, H, R = 3840, 2160, a.range
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    nf = 8
    p0, _ = xd.frame_shard(world * nf, world, rank)
    luma, stride, origin, nv, cs, co = synth.make_subpel_sequence(nf + 1, W, H, 8, start=p0)
    pad, cpad = synth.PAD, 16
    # the pictures: unpadded planes in pinned memory (x264_picture_t's planes)
    host_y = torch.from_numpy(np.ascontiguousarray(luma[:, pad:pad + H, pad:pad + W])).pin_memory()
    host_c = torch.from_numpy(np.ascontiguousarray(nv[:, cpad:cpad + H // 2, 2 * cpad:2 * cpad + W])).pin_memory()
    up_bytes = (host_y[0].numel() + host_c[0].numel())
    fsz, csz = luma[0].size, nv[0].size
    del luma, nv
    ring = torch.empty((3, H + 2 * pad, stride), dtype=torch.uint8, device="cuda")
    cring = torch.empty((3, H // 2 + 2 * cpad, cs), dtype=torch.uint8, device="cuda")
    hp = [[torch.empty_like(ring[0:1]) for _ in range(3)] for _ in range(3)]
    par, init, cm, span = tesa_params(mbw, mbh, 1, R, centre=(0, 0))
    par_d, init_d = torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda()
    cm_d = torch.from_numpy(cm.view(np.int16)).cuda()
    dec = torch.empty((nmb, 3), dtype=torch.int32, device="cuda")
    mb = np.arange(nmb)
    mbx, mby = mb % mbw, mb // mbw
    pos_d = torch.from_numpy(np.stack([0 * mb, 16 * mbx, 16 * mby], 1).astype(np.int32)).cuda()
    rpar = np.zeros((nmb, 8), np.int16)
    rpar[:, 4], rpar[:, 5] = 4 * (-16 * mbx - 24), 4 * (-16 * mby - 24)
    rpar[:, 6], rpar[:, 7] = 4 * (16 * (mbw - 1 - mbx) + 24), 4 * (16 * (mbh - 1 - mby) + 24)
    rpar_d = torch.from_numpy(rpar).cuda()
    rinit = torch.empty(nmb, dtype=torch.int32, device="cuda")
    rout = torch.empty((nmb, 4), dtype=torch.int32, device="cuda")
    ne = torch.empty(nmb, dtype=torch.int32, device="cuda")
    flat = [16] * 64
    q4m, q4b, _, _ = x.cqm_init(8, [flat] * 8)
    mf4 = torch.from_numpy(q4m[1, 26].copy()).cuda()
    bs4 = torch.from_numpy(q4b[1, 26].copy()).cuda()
    dct = torch.empty((nmb, 256), dtype=torch.int16, device="cuda")
    nz = torch.empty(nmb, dtype=torch.int32, device="cuda")
    # chroma ME inputs per (cur, ref) ring pair (x264hip_refine_ext_t), built once
    exts = {(c, r): x.refine_ext(1, 1, 0, fenc_chroma=[cring[c:c + 1]], fenc_chroma_origin=co, fenc_chroma_stride=cs,
                                 ref_chroma=[cring[r:r + 1]], ref_chroma_origin=co, ref_chroma_stride=cs)
            for c in range(3) for r in range(3) if c != r}

    # one x264hip_upload_planes launch per picture (luma + NV12), its records built once
    ups = {(slot, i): [x.plane_upload(ring[slot], origin, stride, host_y[i], unit=1, pad_x=pad, pad_y=pad),
                       x.plane_upload(cring[slot], co, cs, host_c[i], unit=2, pad_x=2 * cpad, pad_y=cpad)]
           for slot in range(3) for i in range(nf + 1)}

    def upload(slot, i):
        x.upload_planes(ups[(slot, i)])

    def esa(cur, ref):
        """the exhaustive search of me.c:618-631 over range R around mv 0 with its decision, fused
        (x264hip_8_me_search_esa: the SAD table never leaves the chip)"""
        x.me_search_esa(cur, origin, stride, ref, origin, stride, mbw, mbh, 1, R, R, par_d, init_d, (cm_d, span),
                        out=dec, fenc_frame_stride=fsz, ref_frame_stride=fsz)

    def frame(c, r):
        """the compute of one frame: ring slot c against slot r (r's hpel planes already built)"""
        cur, ref = ring[c:c + 1], ring[r:r + 1]
        x.hpel_filter(cur, origin, stride, W, H, outs=hp[c])
        esa(cur, ref)
        rpar_d[:, 0:2] = dec[:, 1:3] * 4
        rinit.copy_(dec[:, 0])
        x.me_refine_subpel(cur, origin, stride, [ref] + hp[r], origin, stride, x.PIXEL_16x16, 7, pos_d, rpar_d,
                           rinit, (cm_d, span), out=rout, fenc_frame_stride=fsz, ref_frame_stride=fsz, nevals=ne,
                           ext=exts[(c, r)])
        x.mb_dct_quant(4, cur, origin, stride, ref, origin, stride, mbw, mbh, 1, mf4, bs4, dct=dct, nz=nz,
                       fenc_frame_stride=fsz, pred_frame_stride=fsz)

    # the refine's candidates per frame pair of the shard (the same pairs the timed steps cycle)
    upload(0, 0)
    x.hpel_filter(ring[0:1], origin, stride, W, H, outs=hp[0])
    rcands, rchroma, moved = [], [], []
    for i in range(nf):
        c, r = (i + 1) % 3, i % 3
        upload(c, i + 1)
        frame(c, r)
        rcands.append(int((ne & 0xFFFF).sum().item()) + int(((ne >> 16) & 0xFF).sum().item()))
        rchroma.append(int((ne >> 24).sum().item()))
        moved.append((rout[:, 1:3] != rpar_d[:, 0:2].int()).any(1).float().mean().item())
    cand_frame = nmb * (2 * R + 1) ** 2 + float(np.mean(rcands))

    comp, copy = x.stream_pair(16)
    done = [torch.cuda.Event() for _ in range(3)]
    ready = [torch.cuda.Event() for _ in range(3)]
    state = {"n": 0}

    def step():
        n = state["n"]
        c, r = (n + 1) % 3, n % 3
        with torch.cuda.stream(copy):                 # upload frame n+1 while frame n's kernels may still run
            copy.wait_event(done[c])
            upload(c, (n + 1) % (nf + 1))
            ready[c].record(copy)
        with torch.cuda.stream(comp):
            comp.wait_event(ready[c])
            frame(c, r)
            done[r].record(comp)
        state["n"] = n + 1

    def reset():
        torch.cuda.synchronize()
        state["n"] = 0
        upload(0, 0)
        x.hpel_filter(ring[0:1], origin, stride, W, H, outs=hp[0])
        for ev in ready + done:
            ev.record()
        torch.cuda.synchronize()
    reset()
    cur_stream = torch.cuda.current_stream()
    wall, _ = timed(step, a.steps, a.warmup, world)
    cur_stream.wait_stream(comp)
    # the parts alone: the upload (both planes) and the compute of one frame
    reset()
    with torch.cuda.stream(copy):
        _, up_ms = timed(lambda: upload(1, 1), a.steps, min(a.warmup, 20), world)
    with torch.cuda.stream(comp):
        _, comp_ms = timed(lambda: frame(1, 0), a.steps, min(a.warmup, 20), world)
    # host time to enqueue one step (no GPU wait inside step())
    reset()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    host_ms = (time.perf_counter() - t0) / a.steps * 1e3
    torch.cuda.synchronize()
    value = world * a.steps * cand_frame / wall
    # the dominant kernel alone (the fused search + decision of one 2160p frame) on the compute
    # stream's 240 CUs, events on that stream
    with torch.cuda.stream(comp):
        _, s_ms = timed(lambda: esa(ring[1:2], ring[0:1]), a.steps, a.warmup, world)
    torch.cuda.synchronize()
    x.stream_pair_destroy((comp, copy))
    absd = nmb * (2 * R + 1) ** 2 * 256
    roof = {"kernel": "me_full_esa_v7_kernel<%d, false>" % R, "bound": "valu",
            "achieved": absd / (s_ms * 1e-3) / 1e12, "peak": SAD_PEAK_ABSDIFF / 1e12,
            "unit": "T byte-absdiff/s (algorithmic: 256 per 16x16 candidate)",
            "frac": absd / (s_ms * 1e-3) / SAD_PEAK_ABSDIFF, "traffic": None, "launch_ms": s_ms,
            "cus": 240, "peak_note": "peak is the whole chip's 256 CUs; the kernel runs on the compute stream's 240",
            "algorithmic_bytes_per_launch": 2 * nmb * 256 + nmb * 12}
    ms = wall / a.steps * 1e3
    out = {
        "metric": "SAD+SATD candidate-MVs/sec + DCT+quant blocks/sec, 1080p, 1/2/4/8 GPU",
        "value": value,
        "unit": "candidate MVs/s (SAD16x16 full-search table + refine_subpel SAD/SATD calls)",
        "n_gpus": pg_world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "configs[3]: 3840x2160 4:2:0, full-search ME range %d (fused search + ESA decision) + "
                               "refine_subpel subme 7 with chroma ME (SAD/SATD + U/V SATD) + 4x4 DCT/quant per "
                               "frame, one frame per GPU per step uploaded from pinned host pictures (luma + "
                               "NV12, borders expanded on the way in; H2D in the timed region)" % R,
                   "content": "synth.make_subpel_sequence: quarter-pel motion (3.25, 2.5) px per frame",
                   "b_chroma_me": 1, "frames_per_step_per_gpu": 1, "mbs_per_frame": nmb,
                   "candidates_per_mb": cand_frame / nmb, "table_candidates_per_mb": (2 * R + 1) ** 2,
                   "refine_candidates_per_frame": float(np.mean(rcands)),
                   "refine_chroma_calls_per_frame": float(np.mean(rchroma)),
                   "refine_moved_frac": float(np.mean(moved)), "upload_bytes_per_frame": int(up_bytes),
                   "upload_ms": up_ms, "upload_GBps": up_bytes / (up_ms * 1e-3) / 1e9, "compute_ms": comp_ms,
                   "host_enqueue_ms": host_ms, "step_vs_upload": ms / up_ms,
                   "parallelism": "frame-per-GPU x%d" % world, "world_size": pg_world, "rank_devices": rank_dev,
                   "dist_backend": (os.environ.get("X264HIP_DIST_BACKEND", "nccl") if world > 1 else None)},
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as orc  # cpu_baseline leg only
        f0 = ring[1].cpu().numpy().ravel()
        f1 = ring[0].cpu().numpy().ravel()
        try:
            share = len(os.sched_getaffinity(0))
        except AttributeError:
            share = os.cpu_count() or 1
        nthr = min(16, share)
        band = 16                                     # MB rows of the sample per call
        t0, calls = time.perf_counter(), 0
        while True:
            orc.me_search_full_mt(f0, origin, stride, f1, origin, stride, mbw, band, R, nthr)
            calls += 1
            if time.perf_counter() - t0 >= a.cpu_seconds:
                break
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": calls * mbw * band * (2 * R + 1) ** 2 / dt, "unit": "SAD16x16 candidates/s",
                               "cores": nthr, "kind": "port", "cpu_model": cpu_model(),
                               "sample": "%d calls of the full search over %d of the frame's %d MB rows, %d "
                                         "threads, %.1f s" % (calls, band, mbh, nthr, dt)}
    del ring, cring, hp, host_y, host_c
    return out


def parse():
    ap = argparse.ArgumentParser()
    # N ranks, one per GPU: started here as child processes when no launcher set WORLD_SIZE
    ap.add_argument("--gpus", type=int, default=None)
    # the GPU's clocks settle only after ~100 back-to-back launches (~35 ms of load,
    # tools/me_sustain.py: 0.35-0.40 ms per launch at first, 0.306 ms steady), so the
    # default warmup covers the ramp; every step is still a full launch over F pairs
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=150)
    # 128 pairs per headline step: a 2.2-ms launch, so the driver's 5 warmup steps carry the
    # GPU through most of its ~20-ms clock transient (profiles/r03a_trace_*: after an idle gap
    # the first launches of a 16-pair step ran 12-30 % slow).  Under the driver's arguments
    # (--steps 20 --warmup 5): 16 pairs 0.65, 64 pairs 0.77, 128 pairs 0.81 of the SAD
    # roofline (profiles/r03l_batch/); steady state is 0.82-0.84 at any batch
    ap.add_argument("--frames", type=int, default=128, help="frame pairs per headline step per GPU")
    ap.add_argument("--xframes", type=int, default=16, help="frame pairs of the side legs (<= --frames)")
    # the streaming transform kernels (DCT+quant, reconstruction) move ~8.5 MB per 1080p
    # frame; SURVEY.md §8d (configs[3]) asks for >= 64 frames per launch so the launch
    # is not dominated by its ramp and tail
    ap.add_argument("--tframes", type=int, default=64, help="frame pairs per transform launch per GPU")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--range", type=int, default=16)
    # configs[1] (the default headline) or configs[3]: a 2160p frame per GPU per step, full search +
    # refine_subpel + DCT/quant, the new frame streamed from pinned host memory (workload_2160p)
    ap.add_argument("--workload", choices=("1080p", "2160p"), default="1080p")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-extra", action="store_true", help="skip the configs[2] side rates")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall-clock bound of the CPU sample")
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # one rank per GPU; X264HIP_DIST_BACKEND=gloo lets several ranks share one GPU
        # to exercise the N > 1 path functionally on a single-GPU box (not a measurement);
        # launch_plan has already refused more RCCL ranks than GPUs
        backend = os.environ.get("X264HIP_DIST_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        dev = local if backend == "nccl" else local % max(1, ndev)
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    from x264hip import dist as xd
    xd.barrier()


def max_over_ranks(v, world):
    from x264hip import dist as xd
    return xd.reduce_max(v, device="cuda")


# extra legs only (set after the headline is measured): keep calling a leg after its
# counted warmup until this much wall time has passed, so a leg of 16-µs launches is not
# timed on clocks that the previous leg's host-side setup let drop (tools/me_sustain.py:
# the clocks need ~35 ms of load to settle); the headline keeps its plain counted warmup
_SETTLE_S = 0.0


def timed(fn, steps, warmup, world, graph=False):
    """Run warmup, then `steps` timed calls bracketed by barrier + synchronize.
    Returns (wall seconds max over ranks, mean per-launch event ms on this rank).

    The mean launch time is one HIP event pair on the launch stream around the `steps`
    back-to-back launches, divided by `steps` (an event between every two launches
    costs ~11 us of command-processor time per step in the kernel trace,
    profiles/r03a_*).  graph=True (extra legs whose launches are shorter than the
    host's per-call overhead, so the queue would drain between Python calls): the
    `steps` calls are captured once into one HIP graph and the timed region is one
    replay of it -- the same launches, without host gaps."""
    if graph:
        try:
            return _timed_graph(fn, steps, warmup, world)
        except RuntimeError as e:                       # capture unsupported: time eagerly
            print("bench.py: graph capture failed (%s); timing eagerly" % e, file=sys.stderr)
            torch.cuda.synchronize()
    for _ in range(warmup):
        fn()
    if _SETTLE_S:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < _SETTLE_S:
            fn()
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    ev_ms = s.elapsed_time(e) / steps
    return max_over_ranks(t1 - t0, world), ev_ms


def _timed_graph(fn, steps, warmup, world):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):                       # allocations made before capture
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(steps):
            fn()
    for _ in range(max(1, warmup // max(1, steps))):
        g.replay()
    if _SETTLE_S:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < _SETTLE_S:
            g.replay()
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    ev_ms = s.elapsed_time(e) / steps
    del g
    return max_over_ranks(t1 - t0, world), ev_ms


def world_devices(world):
    """(process-group world size, the device id of every rank) for the JSON line."""
    dev = torch.cuda.current_device()
    if world == 1:
        return 1, [dev]
    import torch.distributed as dist
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, dev)
    return dist.get_world_size(), got


def main():
    a = parse()
    x = load_package()
    from x264hip import dist as xd0
    try:
        # torch.cuda.device_count() does not initialise HIP, so a launching parent stays
        # GPU-free and its ranks are children (never an exec of a GPU process)
        how, n = xd0.launch_plan(a.gpus, os.environ, torch.cuda.device_count())
    except xd0.LaunchError as e:
        print("bench.py: %s" % e, file=sys.stderr)
        sys.exit(2)
    if how == "spawn":
        rc = xd0.spawn_ranks([os.path.abspath(__file__)] + sys.argv[1:], n, os.environ)
        sys.exit(rc if rc >= 0 else 128 - rc)
    world, rank, local = dist_setup()
    x.init(torch.cuda.current_device())
    pg_world, rank_dev = world_devices(world)
    from x264hip import synth
    if a.workload == "2160p":
        out = workload_2160p(x, a, world, rank, pg_world, rank_dev)
        if rank == 0:
            print(json.dumps(out))
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    W, H, R, F = a.width, a.height, a.range, a.frames
    mbw, mbh = (W + 15) // 16, (H + 15) // 16
    Hp = mbh * 16                                   # x264 pads the height to whole MBs
    cand_per_mb = (2 * R + 1) ** 2
    # one synthetic sequence of world*F pairs; pair k = (frame k+1, ref frame k);
    # rank r owns pairs [r*F, (r+1)*F) and builds only frames r*F .. r*F+F
    from x264hip import dist as xd
    p0, p1 = xd.frame_shard(world * F, world, rank)
    planes, stride, origin = synth.make_sequence(p1 - p0 + 1, W, Hp, 8, start=p0)
    dev = torch.from_numpy(planes).cuda()
    fstride = planes[0].size
    table = torch.empty((F, mbh, mbw, 2 * R + 1, x.me_table_pitch(R)), dtype=torch.int16, device="cuda")

    def step():
        x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, R, table=table,
                         fenc_frame_stride=fstride, ref_frame_stride=fstride)

    wall, ev_ms = timed(step, a.steps, a.warmup, world)
    cands = world * a.steps * F * mbw * mbh * cand_per_mb
    value = cands / wall
    ms_per_step = wall / a.steps * 1e3
    global _SETTLE_S
    _SETTLE_S = 0.04

    # roofline of the dominant kernel (me_full_sad16): algorithmic absdiffs per launch
    absdiff_per_launch = F * mbw * mbh * cand_per_mb * 256
    achieved = absdiff_per_launch / (ev_ms * 1e-3)
    roof = {
        # the launched template: <range, table pitch in dwords> (me.hip launch_me_full)
        "kernel": "me_full_sad16_v7_kernel<%d, %d>" % (R, x.me_table_pitch(R) // 4),
        "bound": "valu",
        "achieved": achieved / 1e12,
        "peak": SAD_PEAK_ABSDIFF / 1e12,
        "unit": "T byte-absdiff/s (algorithmic: 256 per 16x16 candidate)",
        "frac": achieved / SAD_PEAK_ABSDIFF,
        "traffic": None,
        "algorithmic_bytes_per_launch": F * (mbw * mbh * 256 + mbw * mbh * 256 + mbw * mbh * cand_per_mb * 2),
        "launch_ms": ev_ms,
    }
    # HBM bytes per launch from the newest committed PMC summary (tools/gpu_profile.sh +
    # tools/pmc_summarize.py: separate FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected),
    # used only when it profiled this kernel on this workload
    import glob
    def _tag_order(path):
        # round tags rNNx..: r03z < r03aa < r03ab (one letter runs out before two)
        t = os.path.basename(path).split("_")[0]
        return (t[:3], len(t), t)
    pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")), key=_tag_order)
    if pmcs:
        with open(pmcs[-1]) as fh:
            d = json.load(fh)
        if (d.get("frames") == F and d.get("range") == R and d.get("width") == W
                and d.get("trace", {}).get("kernel") == roof["kernel"].split("<")[0]):
            roof["traffic"] = d.get("hbm_bytes_per_launch")
            roof["traffic_source"] = os.path.relpath(pmcs[-1], ROOT)

    out = {
        "metric": "SAD+SATD candidate-MVs/sec + DCT+quant blocks/sec, 1080p, 1/2/4/8 GPU",
        "value": value,
        "unit": "SAD16x16 candidates/s",
        "n_gpus": pg_world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": "configs[1]: %dx%d luma, full-search ME range %d, sad_16x16 candidate tables, "
                               "%d frame pairs per GPU per step" % (W, H, R, F),
                   "frames_per_step_per_gpu": F, "mbs_per_frame": mbw * mbh, "candidates_per_mb": cand_per_mb,
                   "parallelism": "frame-per-GPU x%d" % world,
                   "world_size": pg_world, "rank_devices": rank_dev,
                   "dist_backend": (os.environ.get("X264HIP_DIST_BACKEND", "nccl") if world > 1 else None)},
        "roofline": roof,
    }

    if not a.no_extra:
        XF = min(a.xframes, F)
        out["extra"] = extra_rates(x, a, world, dev[:XF + 1], origin, stride, fstride, mbw, mbh, XF, full=dev)
        # the headline kernel again after the extra legs have kept the GPU busy for tens of
        # seconds: its steady-state launch time and roofline fraction, reported beside (never
        # instead of) the timed region above, which starts after only --warmup launches
        _, ss_ms = timed(step, a.steps, 10, world)
        out["extra"]["me_steady_launch_ms"] = ss_ms
        out["extra"]["me_steady_frac"] = absdiff_per_launch / (ss_ms * 1e-3) / SAD_PEAK_ABSDIFF
    if rank == 0 and world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(planes, origin, stride, mbw, mbh, R, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def extra_rates(x, a, world, dev, origin, stride, fstride, mbw, mbh, F, full=None):
    """configs[2] side rates on the same frames: SATD 8x8 candidates/s and fused
    DCT+quant blocks/s (QP 26, flat16 CQM, inter-luma lists, zero-MV prediction)."""
    # configs[3]'s streaming leg first: after any leg that captured and replayed a HIP graph,
    # this process's two-stream upload / search overlap measured ~25 % slower (0.175 -> 0.22 ms
    # per 2160p frame whichever graph-timed leg ran before it, GPU_MAX_HW_QUEUES 4, 8 or 16
    # alike; profiles/r03o_after.log, r03p_after.log) -- a runtime interaction not isolated
    # further, noted in DESIGN.md §6
    r2160 = rates_2160p(x, a, world)
    res = {}
    flat = [16] * 64
    q4m, q4b, q8m, q8b = x.cqm_init(8, [flat] * 8)
    mf4 = torch.from_numpy(q4m[1, 26].copy()).cuda()
    bs4 = torch.from_numpy(q4b[1, 26].copy()).cuda()
    mf8 = torch.from_numpy(q8m[1, 26].copy()).cuda()
    bs8 = torch.from_numpy(q8b[1, 26].copy()).cuda()
    # transform legs: their own TF-pair shard of the same sequence (>= 64 frames per launch)
    from x264hip import synth, dist as xd
    TF = a.tframes
    t0, t1 = xd.frame_shard(world * TF, world, int(os.environ.get("RANK", "0")))
    tplanes, _, _ = synth.make_sequence(t1 - t0 + 1, mbw * 16, mbh * 16, 8, start=t0)
    tdev = torch.from_numpy(tplanes).cuda()
    del tplanes
    # the prediction as a buffer of its own (an encoder's motion-compensated prediction is not
    # the previous source frame): as slices of one sequence every frame would be read twice,
    # once as a source and once as a prediction, and the second read served from cache
    tpred = tdev[:-1].clone()
    nmb = TF * mbw * mbh
    dct = torch.empty((nmb, 256), dtype=torch.int16, device="cuda")
    nz = torch.empty(nmb, dtype=torch.int32, device="cuda")
    for t, mf, bs in ((4, mf4, bs4), (8, mf8, bs8)):
        def step(t=t, mf=mf, bs=bs):
            x.mb_dct_quant(t, tdev[1:], origin, stride, tpred, origin, stride, mbw, mbh, TF, mf, bs, dct=dct,
                           nz=nz, fenc_frame_stride=fstride, pred_frame_stride=fstride)
        wall, ev_ms = timed(step, a.steps, a.warmup, world, graph=True)
        blocks = nmb * (16 if t == 4 else 4)
        bpb = (16 + 16 + 32) if t == 4 else (64 + 64 + 128)     # fenc + pred in, int16 coefs out
        res["dct%d_quant_blocks_per_s" % t] = world * a.steps * blocks / wall
        res["dct%d_quant_hbm_frac" % t] = blocks * bpb / (ev_ms * 1e-3) / HBM_PEAK
        res["dct%d_quant_launch_ms" % t] = ev_ms
    # SATD 8x8 subpel refine (configs[2]): half-pel planes of the F refs, then for every
    # 8x8 block 9 quarter-pel candidates (+-1 qpel) around a half-pel MV next to the true
    # motion (3, 2) px, each an unweighted get_ref + satd_8x8 (reference me.c:950-963)
    hv = [torch.zeros_like(dev) for _ in range(3)]

    def hstep():
        x.hpel_filter(dev[:-1], origin, stride, mbw * 16, mbh * 16, outs=[h[:-1] for h in hv])
    wall, ev_ms = timed(hstep, a.steps, a.warmup, world, graph=True)
    res["hpel_filter_frames_per_s"] = world * a.steps * F / wall
    res["hpel_filter_launch_ms"] = ev_ms
    # algorithmic bytes: the padded source plane in, the three padded half-pel planes out
    res["hpel_filter_hbm_frac"] = F * 4 * dev[0].numel() / (ev_ms * 1e-3) / HBM_PEAK
    # fused reconstruction (dequant + idct + add, per-MB qp) on the coefficients of the last
    # DCT+quant step, and the lookahead's half-resolution planes
    dq4, dq8 = x.cqm_dequant([flat] * 8)
    qp_mb = torch.full((nmb,), 26, dtype=torch.int32, device="cuda")
    recon = torch.empty_like(tdev[:-1])
    for t, dq in ((4, dq4[1]), (8, dq8[1])):
        x.mb_dct_quant(t, tdev[1:], origin, stride, tdev[:-1], origin, stride, mbw, mbh, TF,
                       mf4 if t == 4 else mf8, bs4 if t == 4 else bs8, dct=dct, nz=nz,
                       fenc_frame_stride=fstride, pred_frame_stride=fstride)
        dqd = torch.from_numpy(dq.copy()).cuda()

        def rstep(t=t, dqd=dqd):
            x.mb_dequant_idct_add(t, dct, mbw, mbh, TF, dqd, qp_mb, tdev[:-1], origin, stride, recon, origin,
                                  stride, pred_frame_stride=fstride, recon_frame_stride=fstride)
        wall, ev_ms = timed(rstep, a.steps, a.warmup, world, graph=True)
        blocks = nmb * (16 if t == 4 else 4)
        bpb = (32 + 16 + 16) if t == 4 else (128 + 64 + 64)      # int16 coefs + pred in, recon out
        res["recon%d_blocks_per_s" % t] = world * a.steps * blocks / wall
        res["recon%d_hbm_frac" % t] = blocks * bpb / (ev_ms * 1e-3) / HBM_PEAK
        res["recon%d_launch_ms" % t] = ev_ms
    # the two streaming frame kernels at the transform legs' batch (>= 64 frames per
    # launch), where the launch ramp and tail no longer dominate
    fb = tdev[0].numel()
    thv = [torch.empty_like(tdev[:-1]) for _ in range(3)]

    def h64():
        x.hpel_filter(tdev[:-1], origin, stride, mbw * 16, mbh * 16, outs=thv)
    wall, ev_ms = timed(h64, a.steps, a.warmup, world, graph=True)
    res["hpel_filter_%d_frames_per_s" % TF] = world * a.steps * TF / wall
    res["hpel_filter_%d_launch_ms" % TF] = ev_ms
    res["hpel_filter_%d_hbm_frac" % TF] = TF * 4 * fb / (ev_ms * 1e-3) / HBM_PEAK
    del thv
    tl, _ = x.frame_init_lowres(tdev[:-1], origin, stride, mbw * 16, mbh * 16)

    def l64():
        x.frame_init_lowres(tdev[:-1], origin, stride, mbw * 16, mbh * 16, outs=tl)
    wall, ev_ms = timed(l64, a.steps, a.warmup, world, graph=True)
    lbytes = fb + 4 * tl[0][0].numel()              # source plane in, four padded lowres planes out
    res["lowres_%d_frames_per_s" % TF] = world * a.steps * TF / wall
    res["lowres_%d_launch_ms" % TF] = ev_ms
    res["lowres_%d_hbm_frac" % TF] = TF * lbytes / (ev_ms * 1e-3) / HBM_PEAK
    del tl
    del recon, tdev, tpred, dct, nz
    lw, lh = mbw * 16, mbh * 16
    louts, _ = x.frame_init_lowres(dev[:-1], origin, stride, lw, lh)

    def lstep():
        x.frame_init_lowres(dev[:-1], origin, stride, lw, lh, outs=louts)
    wall, ev_ms = timed(lstep, a.steps, a.warmup, world, graph=True)
    res["lowres_frames_per_s"] = world * a.steps * F / wall
    res["lowres_launch_ms"] = ev_ms
    res["lowres_hbm_frac"] = F * (dev[0].numel() + 4 * louts[0][0].numel()) / (ev_ms * 1e-3) / HBM_PEAK
    # the lookahead's intra estimate on those lowres planes (slicetype.c:714-757, subme > 1:
    # 10 predictions + satd_8x8 per 8x8 block, lambda of X264_LOOKAHEAD_QP = 12 -> 1, slicetype.c:47-48)
    iouts = x.lowres_intra_cost(louts[0], x.plane_stride(lw // 2), mbw, mbh, True, True, 1)

    def istep():
        x.lowres_intra_cost(louts[0], x.plane_stride(lw // 2), mbw, mbh, True, True, 1, outs=iouts)
    wall, ev_ms = timed(istep, a.steps, a.warmup, world, graph=True)
    res["lowres_intra_mbs_per_s"] = world * a.steps * F * mbw * mbh / wall
    res["lowres_intra_launch_ms"] = ev_ms
    res.update(rates_lookahead(x, a, world, louts, iouts, lw, mbw, mbh, F))
    del louts, iouts
    res.update(rates_weightp(x, a, world, dev, origin, stride, mbw, mbh))
    res.update(rates_ssim(x, a, world, dev, origin, stride, mbw, mbh))
    nb8 = mbw * mbh * 4
    ys, xs = np.meshgrid(np.arange(mbh * 2), np.arange(mbw * 2), indexing="ij")
    bx, by = (xs.ravel() * 8).astype(np.int64), (ys.ravel() * 8).astype(np.int64)
    # one entry per 8x8 block: its half-pel centre (3.5, 2) px; the nine candidates are the
    # +-1 quarter-pel neighbourhood (subpel_qpel9_batch); the same candidates as a flat
    # list (one lane per candidate, subpel_cmp_batch) are timed beside it
    bfo, cxy, fo, qxy = [], [], [], []
    for f in range(F):
        bfo.append((f + 1) * fstride + origin + by * stride + bx)
        c = np.stack([4 * bx + 12 + 2, 4 * by + 8 + 4 * f * (fstride // stride)], 1)
        cxy.append(c.astype(np.int32))
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                fo.append(bfo[-1])
                qxy.append((c + np.array([dx, dy])).astype(np.int32))
    bfo = torch.from_numpy(np.concatenate(bfo)).cuda()
    cxy = torch.from_numpy(np.concatenate(cxy)).cuda()
    fo = torch.from_numpy(np.concatenate(fo)).cuda()
    qxy = torch.from_numpy(np.concatenate(qxy)).cuda()
    sc = torch.empty(fo.numel(), dtype=torch.int32, device="cuda")
    sc9 = torch.empty((bfo.numel(), 9), dtype=torch.int32, device="cuda")
    flat = dev.view(-1)
    ref_planes = [dev.view(-1)] + [h.view(-1) for h in hv]

    def s9step():
        x.subpel_qpel9_batch(x.CMP_SATD, x.PIXEL_8x8, flat, stride, ref_planes, origin, stride, bfo, cxy, scores=sc9)
    wall, ev_ms = timed(s9step, a.steps, a.warmup, world, graph=True)
    cands = sc9.numel()
    res["satd8x8_subpel_candidates_per_s"] = world * a.steps * cands / wall
    res["satd8x8_subpel_launch_ms"] = ev_ms
    res["satd8x8_candidates_per_launch"] = int(cands)
    # 444 lane-ops per SATD 8x8 + 192 for the qpel averages, vs the VALU peak
    res["satd8x8_subpel_frac"] = cands * (444 + 192) / (ev_ms * 1e-3) / VALU_LANE_OPS

    def sstep():
        x.subpel_cmp_batch(x.CMP_SATD, x.PIXEL_8x8, flat, stride, ref_planes, origin, stride, fo, qxy, scores=sc)
    wall, ev_ms = timed(sstep, a.steps, a.warmup, world, graph=True)
    res["satd8x8_subpel_list_candidates_per_s"] = world * a.steps * fo.numel() / wall
    res["satd8x8_subpel_list_launch_ms"] = ev_ms
    # both entries score the same candidates (list order: frame, dy, dx, block)
    nbl = bx.size
    lst = sc.view(F, 9, nbl).permute(0, 2, 1).reshape(-1, 9)
    if not torch.equal(lst, sc9):
        raise SystemExit("bench: subpel_qpel9_batch and subpel_cmp_batch disagree")
    del nb8, hv, ref_planes, fo, qxy, sc, bfo, cxy, sc9, lst
    res.update(rates_tesa(x, a, world, dev, origin, stride, fstride, mbw, mbh, F))
    # plane SSD is a streaming reduction: timed at the streaming kernels' >= 64 frames per
    # launch when the headline batch holds them, and at F beside it
    res.update(rates_ssd(x, a, world, dev, origin, stride, F))
    if full is not None and full.shape[0] - 1 >= a.tframes:
        r64 = rates_ssd(x, a, world, full[:a.tframes + 1], origin, stride, a.tframes)
        res.update({k.replace("ssd_plane", "ssd_plane_%d" % a.tframes): v for k, v in r64.items()})
    res.update(rates_esa(x, a, world, dev, origin, stride, fstride, mbw, mbh, F))
    res.update(rates_refine(x, a, world, mbw, mbh, F))
    res.update(rates_full8(x, a, world, dev, origin, stride, fstride, mbw, mbh, F))
    res.update(rates_esa8(x, a, world, dev, origin, stride, fstride, mbw, mbh, F))
    res.update(rates_10bit(x, a, world, mbw, mbh, F))
    res.update(r2160)
    return res


def tesa_params(mbw, mbh, F, R, centre=(-3, -2)):
    """TESA search parameters of every MB of F frames: the window centred on a predictor
    next to the synthetic motion, mv_limit_fpel-shaped limits (analyse.c:330-349), mvp =
    the centre, no predictor cost to beat; an x264-shaped cost_mv table (lambda 4)."""
    n1 = mbw * mbh
    mb = np.arange(F * n1) % n1
    mbx, mby = mb % mbw, mb // mbw
    par = np.zeros((F * n1, 8), np.int16)
    par[:, 0], par[:, 1] = centre
    par[:, 2], par[:, 3] = 4 * centre[0], 4 * centre[1]
    par[:, 4], par[:, 5] = -16 * mbx - 24, -16 * mby - 24
    par[:, 6], par[:, 7] = 16 * (mbw - 1 - mbx) + 20, 16 * (mbh - 1 - mby) + 24
    init = np.full(F * n1, 1 << 30, np.int32)
    span = 16384
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    cm = np.minimum((4 * logs + 0.5).astype(np.int64), 65535).astype(np.uint16)
    return par, init, cm, span


def lookahead_cost_mv():
    """cost_mv[X264_LOOKAHEAD_QP] over +-8*512 (analyse.c:143-157, lambda 1): (device table, mvd-0 index)"""
    span = 8 * 512
    ii = np.arange(span + 1, dtype=np.float32)
    logs = np.where(ii == 0, np.float32(0.718), np.log2(ii + np.float32(1)) * np.float32(2) + np.float32(1.718))
    half = np.minimum((logs.astype(np.float32) + np.float32(0.5)).astype(np.int64), 65535).astype(np.uint16)
    return torch.from_numpy(np.concatenate([half[:0:-1], half]).view(np.int16)).cuda(), span


def rates_weightp(x, a, world, dev, origin, stride, mbw, mbh):
    """x264_weights_analyse (slicetype.c:284-501) on a fade of the bench's first frame pair (frame 1
    scaled by 0.85, +12; the bench sequence is luma only): the lookahead's call (the guessed weight
    and the weighted lowres plane, slicetype.c:859-862) and the encoder's call at subme 7 with the
    pair's lowres mvs (slicetype.c:1939-1943).  Each call is synchronous (one batch of candidate
    costs, a stream synchronise, the host's replay of the search): per-call wall time.  Beside it
    the frame statistics kernel (ac_energy_mb's sums, ratecontrol.c:225-257) per 1080p frame."""
    W, H = mbw * 16, mbh * 16
    fade = (dev[1].float() * 0.85 + 12).round().clamp(0, 255).to(torch.uint8)
    pair = torch.stack([dev[0], fade])
    louts, ls = x.frame_init_lowres(pair, origin, stride, W, H)
    intra = x.lowres_intra_cost(louts[0][1:], ls, mbw, mbh, True, True, 1)[0]
    st = torch.empty(6, dtype=torch.int64, device="cuda")

    def sstep():
        x.frame_pixel_stats(pair[1], origin, stride, mbw, mbh, out=st)
    wall, ev_ms = timed(sstep, a.steps, a.warmup, world, graph=True)
    res = {"pixel_stats_frames_per_s": world * a.steps / wall, "pixel_stats_launch_ms": ev_ms}
    stats = []
    for i in range(2):
        v = x.frame_pixel_stats(pair[i], origin, stride, mbw, mbh).cpu().numpy().view(np.uint64)
        stats.append(([int(t) for t in v[:3]], [int(t) for t in v[3:]]))
    cm, span = lookahead_cost_mv()
    mvs = x.lowres_inter_cost(louts[0][1:], [p[:1] for p in louts], ls, mbw, mbh, intra, (cm, span))[0][0]
    wl = torch.zeros_like(louts[0][0])
    fl, rl = louts[0][1], [p[0] for p in louts]
    for name, kw in (("la", dict(b_lookahead=True, weighted_lowres=wl)),
                     ("enc", dict(b_lookahead=False, subme=7, mvs=mvs))):
        w = None

        def wstep(kw=kw):
            nonlocal w
            w = x.weights_analyse(fl, rl, ls, mbw, mbh, intra[0], stats[1], stats[0], **kw)
        wall, _ = timed(wstep, max(1, a.steps // 2), 2, world)
        res["weightp_%s_ms" % name] = wall / max(1, a.steps // 2) * 1e3
        res["weightp_%s_weight" % name] = list(w[0][0])
    return res


def rates_ssim(x, a, world, dev, origin, stride, mbw, mbh):
    """x264_pixel_ssim_wxh (pixel.c:690-714) of 1080p frame pairs: as the encoder calls it, once
    per filtered MB-row band (encoder.c:2412-2420, 2516-2528; 68 bands per frame, each band's
    float independent), batched by x264hip_*_ssim_bands -- one frame per launch (ssim_bands_*)
    and every frame of the batch in one launch (ssim_bands_batch_*) -- and, beside it, the whole
    frame as one x264_pixel_ssim_wxh call (ssim_*: one ordered float chain).  Frames per second
    including the ordered float sums; per-frame input 2 x 1920 x 1088 bytes."""
    W, H = mbw * 16, mbh * 16
    cnt = [0]
    F = dev.shape[0] - 1
    hgt = min(H, a.height)

    def step():
        cnt[0] = x.ssim_wxh(dev[1], origin + 2, stride, dev[0], origin + 2, stride, W - 2, H)[1]
    wall, _ = timed(step, max(1, a.steps // 2), 2, world)
    n = max(1, a.steps // 2)
    res = {"ssim_frames_per_s": world * n / wall, "ssim_ms": wall / n * 1e3, "ssim_windows": cnt[0]}
    bands = torch.from_numpy(x.ssim_encoder_bands(mbh, hgt)).cuda()
    out1 = torch.empty((1, bands.shape[0]), dtype=torch.float32, device="cuda")
    outb = torch.empty((F, bands.shape[0]), dtype=torch.float32, device="cuda")

    def bstep():
        x.ssim_bands(dev[1:2], origin + 2, stride, dev[0:1], origin + 2, stride, W - 2, bands, out=out1)

    def fstep():
        x.ssim_bands(dev[1:], origin + 2, stride, dev[:-1], origin + 2, stride, W - 2, bands, out=outb)
    wall, ev_ms = timed(bstep, a.steps, a.warmup, world, graph=True)
    res.update({"ssim_bands_frames_per_s": world * a.steps / wall, "ssim_bands_launch_ms": ev_ms,
                "ssim_bands_per_frame": int(bands.shape[0])})
    wall, ev_ms = timed(fstep, a.steps, a.warmup, world, graph=True)
    res.update({"ssim_bands_batch_frames_per_s": world * a.steps * F / wall, "ssim_bands_batch_launch_ms": ev_ms,
                "ssim_bands_batch_frames": F,
                "ssim_bands_batch_hbm_frac": F * 2 * W * hgt / (ev_ms * 1e-3) / HBM_PEAK})
    return res


def rates_lookahead(x, a, world, louts, iouts, lw, mbw, mbh, F):
    """The lookahead's lowres motion searches over the F lowres frames (frame_init_lowres
    planes louts, intra costs iouts): P pairs (1, 4 and 8 slices, and a 240-pair batch) and
    B triplets."""
    res = {}
    # the lookahead's P-frame lowres motion search on the same planes: frame k+1 against
    # frame k for the F-1 pairs, HEX + subme 4 (lowres_context_init for subme > 1), range 16,
    # lambda 1, cost_mv[X264_LOOKAHEAD_QP] over +-8*512 (analyse.c:143-157)
    cm, span = lookahead_cost_mv()
    lref = [p[:-1] for p in louts]
    lint = iouts[0][1:]
    louts2 = x.lowres_inter_cost(louts[0][1:], lref, x.plane_stride(lw // 2), mbw, mbh, lint, (cm, span))

    def lastep():
        x.lowres_inter_cost(louts[0][1:], lref, x.plane_stride(lw // 2), mbw, mbh, lint, (cm, span), outs=louts2,
                            check=False)
    # (the lookahead launches are asynchronous: the wavefront status is checked after each leg)
    wall, ev_ms = timed(lastep, max(1, a.steps // 5), max(1, a.warmup // 10), world)
    x.lowres_status()
    res["lowres_me_pairs_per_s"] = world * max(1, a.steps // 5) * (F - 1) / wall
    res["lowres_me_launch_ms"] = ev_ms
    res["lowres_me_pairs_per_launch"] = F - 1
    # the same search as x264 runs it with i_lookahead_threads = T (slicetype.c:901-918): T
    # slices, each its own wavefront (different predictors at slice ends, so different results,
    # as in the reference)
    for T in (4, 8):
        def lsstep(T=T):
            x.lowres_inter_cost(louts[0][1:], lref, x.plane_stride(lw // 2), mbw, mbh, lint, (cm, span), outs=louts2,
                                n_slices=T, check=False)
        wall, ev_ms = timed(lsstep, max(1, a.steps // 5), max(1, a.warmup // 10), world)
        x.lowres_status()
        res["lowres_me_slices%d_pairs_per_s" % T] = world * max(1, a.steps // 5) * (F - 1) / wall
        res["lowres_me_slices%d_launch_ms" % T] = ev_ms
    # the same search at a full-chip batch: 16 copies of those pairs in one launch (one
    # workgroup per pair, 240 of the 256 CUs busy) -- its throughput when the lookahead
    # hands over many (b, p0) pairs at once; the 15-pair leg above is per-pair latency
    nrep = 16
    bf = louts[0][1:].repeat(nrep, 1, 1)
    # the four planes of the references in one buffer, equally spaced (x264's buffer_lowres)
    bb = torch.stack([p[:-1] for p in louts]).repeat(1, nrep, 1, 1)
    br = [bb[k] for k in range(4)]
    bi = lint.repeat(nrep, 1)
    bouts2 = x.lowres_inter_cost(bf, br, x.plane_stride(lw // 2), mbw, mbh, bi, (cm, span))

    def lbstep():
        x.lowres_inter_cost(bf, br, x.plane_stride(lw // 2), mbw, mbh, bi, (cm, span), outs=bouts2, check=False)
    wall, ev_ms = timed(lbstep, max(1, a.steps // 10), 2, world)
    x.lowres_status()
    res["lowres_me_batch_pairs_per_s"] = world * max(1, a.steps // 10) * bf.shape[0] / wall
    res["lowres_me_batch_launch_ms"] = ev_ms
    res["lowres_me_batch_pairs_per_launch"] = int(bf.shape[0])
    del bf, br, bb, bi, bouts2
    # the B-frame leg on the same planes: (p0, b, p1) = (k, k+1, k+2) for the F-2 triplets, both
    # lists searched (a fresh slicetype_frame_cost with b_bidir), p1's list-0 mvs against p0 from
    # one untimed P search as the bidir predictor, equal weights (i_bipred_weight 32, dsf 128)
    ls_ = x.plane_stride(lw // 2)
    nt = F - 2
    nmb_ = mbw * mbh
    p1m = x.lowres_inter_cost(louts[0][2:], [p[:-2] for p in louts], ls_, mbw, mbh, iouts[0][2:], (cm, span))[0]
    bm = [torch.empty((nt, nmb_, 2), dtype=torch.int16, device="cuda") for _ in range(2)]
    bk = [torch.empty((nt, nmb_), dtype=torch.int32, device="cuda") for _ in range(2)]
    bargs = (louts[0][1:-1], [p[:-2] for p in louts], [p[2:] for p in louts], ls_, mbw, mbh, (cm, span), 3,
             bm[0], bk[0], bm[1], bk[1])
    bouts = x.lowres_bidir_cost(*bargs, p1_mvs=p1m)

    def bstep():
        x.lowres_bidir_cost(*bargs, p1_mvs=p1m, outs=bouts, check=False)
    wall, ev_ms = timed(bstep, max(1, a.steps // 5), max(1, a.warmup // 10), world)
    x.lowres_status()
    res["lowres_bidir_triplets_per_s"] = world * max(1, a.steps // 5) * nt / wall
    res["lowres_bidir_launch_ms"] = ev_ms
    res["lowres_bidir_triplets_per_launch"] = nt
    return res


def rates_tesa(x, a, world, dev, origin, stride, fstride, mbw, mbh, F):
    """TESA (me.c:653-748, me_range 16, SATD fpelcmp) over the F 1080p pairs: the
    self-contained form (ads-filtered SADs computed in the kernel) and the form reading
    the headline kernel's full-search table; plus the integral image it needs."""
    R = a.range
    par, init, cm, span = tesa_params(mbw, mbh, F, R)
    par_d, init_d = torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda()
    cm_d = torch.from_numpy(cm.view(np.int16)).cuda()
    H = mbh * 16
    integ = x.frame_integral(dev[:-1], origin, stride, H)

    def istep():
        x.frame_integral(dev[:-1], origin, stride, H, out=integ)
    wall, ev_ms = timed(istep, a.steps, a.warmup, world, graph=True)
    res = {"frame_integral_frames_per_s": world * a.steps * F / wall, "frame_integral_launch_ms": ev_ms}
    out = torch.empty((F * mbw * mbh, 4), dtype=torch.int32, device="cuda")

    def tstep():
        x.me_tesa(dev[1:], origin, stride, dev[:-1], origin, stride, integ, mbw, mbh, F, R, par_d, init_d,
                  (cm_d, span), out=out, fenc_frame_stride=fstride, ref_frame_stride=fstride)
    wall, ev_ms = timed(tstep, a.steps, a.warmup, world)
    res["tesa_mbs_per_s"] = world * a.steps * F * mbw * mbh / wall
    res["tesa_launch_ms"] = ev_ms
    res["tesa_mean_cost_mv_candidates"] = float(out[:, 3].float().mean().item())
    # the search as an encoder would drive it on the GPU: the exhaustive SAD table around each
    # MB's predictor (me_search_centred, the headline kernel) then the TESA scan reading it
    table = torch.empty((F, mbh, mbw, 2 * R + 1, x.me_centred_pitch(8, R)), dtype=torch.int16, device="cuda")
    org = torch.empty((F * mbw * mbh, 2), dtype=torch.int16, device="cuda")
    cen = par_d[:, :2].contiguous()
    out2 = torch.empty_like(out)

    def ttstep():
        x.me_search_centred(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, R, cen, table=table,
                            origin=org, fenc_frame_stride=fstride, ref_frame_stride=fstride)
        x.me_tesa(dev[1:], origin, stride, dev[:-1], origin, stride, integ, mbw, mbh, F, R, par_d, init_d,
                  (cm_d, span), table=table, rng=R, origin=org, out=out2, fenc_frame_stride=fstride,
                  ref_frame_stride=fstride)
    wall, ev_ms = timed(ttstep, a.steps, a.warmup, world)
    res["tesa_centred_table_mbs_per_s"] = world * a.steps * F * mbw * mbh / wall
    res["tesa_centred_table_step_ms"] = ev_ms
    if not torch.equal(out, out2):
        raise SystemExit("bench: me_tesa with and without the SAD table disagree")
    del integ, table, out, out2
    return res


def esa_window_candidates(par, me_range):
    """candidates me.c's ESA evaluates per MB (encoder/me.c:621-631): the clipped window's rows
    times its width rounded as (max_x - min_x + 3) & ~3 -- the algorithmic count the ESA legs'
    fractions are taken on (1056 per unclipped MB at me_range 16: 33 rows x 32 columns)"""
    p = par.astype(np.int64)
    min_x = np.maximum(p[:, 0] - me_range, p[:, 4])
    min_y = np.maximum(p[:, 1] - me_range, p[:, 5])
    max_x = np.minimum(p[:, 0] + me_range, p[:, 6])
    max_y = np.minimum(p[:, 1] + me_range, p[:, 7])
    width = (max_x - min_x + 3) & ~3
    return int((np.maximum(max_y - min_y + 1, 0) * np.maximum(width, 0)).sum())


def rates_esa(x, a, world, dev, origin, stride, fstride, mbw, mbh, F):
    """The ESA decision of every MB of the F pairs (me.c:618-631, window of me_range 16
    centred on the predictor, here mv 0): the table path (the centred search of me.c's
    window, template range = me_range, + me_esa_argmin_at) against the fused kernel that
    never writes the table.  Fractions are taken on the candidates me.c evaluates
    (esa_window_candidates); the template the kernels compute (2R+1 rows x the centred
    pitch, the alignment and width-rounding slack columns included) is reported beside."""
    me_range = a.range
    R = me_range
    par, init, cm, span = tesa_params(mbw, mbh, F, me_range, centre=(0, 0))
    par_d, init_d = torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda()
    cm_d = torch.from_numpy(cm.view(np.int16)).cuda()
    pitch = x.me_centred_pitch(8, R)
    table = torch.empty((F, mbh, mbw, 2 * R + 1, pitch), dtype=torch.int16, device="cuda")
    org = torch.empty((F * mbw * mbh, 2), dtype=torch.int16, device="cuda")
    cen = par_d[:, :2].contiguous()
    out_t = torch.empty((F * mbw * mbh, 3), dtype=torch.int32, device="cuda")
    out_f = torch.empty_like(out_t)

    def search():
        x.me_search_centred(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, R, cen, table=table,
                            origin=org, fenc_frame_stride=fstride, ref_frame_stride=fstride)

    def argmin():
        x.me_esa_argmin(table, R, me_range, par_d, init_d, (cm_d, span), out=out_t, origin=org)

    def tstep():
        search()
        argmin()

    def fstep():
        x.me_search_esa(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, R, me_range, par_d, init_d,
                        (cm_d, span), out=out_f, fenc_frame_stride=fstride, ref_frame_stride=fstride)
    cands = esa_window_candidates(par, me_range)
    tmpl = F * mbw * mbh * (2 * R + 1) * pitch
    wall, ev_ms = timed(tstep, a.steps, a.warmup, world)
    res = {"esa_table_candidates_per_s": world * a.steps * cands / wall, "esa_table_step_ms": ev_ms,
           "esa_template_range": R, "esa_me_range": me_range,
           "esa_window_candidates_per_mb": cands / (F * mbw * mbh),
           "esa_template_candidates_per_mb": tmpl / (F * mbw * mbh)}
    search()
    wall, ev_ms = timed(argmin, a.steps, a.warmup, world, graph=True)
    tbytes = table.numel() * table.element_size()
    res["esa_argmin_launch_ms"] = ev_ms
    res["esa_argmin_table_bytes"] = tbytes
    res["esa_argmin_hbm_frac"] = tbytes / (ev_ms * 1e-3) / HBM_PEAK
    wall, ev_ms = timed(fstep, a.steps, a.warmup, world)
    res["esa_fused_candidates_per_s"] = world * a.steps * cands / wall
    res["esa_fused_step_ms"] = ev_ms
    # SAD roofline on me.c's candidates (256 byte absdiffs each); the template's own rate beside
    res["esa_fused_frac"] = cands * 256 / (ev_ms * 1e-3) / SAD_PEAK_ABSDIFF
    res["esa_fused_template_frac"] = tmpl * 256 / (ev_ms * 1e-3) / SAD_PEAK_ABSDIFF
    if not torch.equal(out_t, out_f):
        raise SystemExit("bench: fused and table ESA decisions disagree")
    del table, org
    return res


def rates_refine(x, a, world, mbw, mbh, F):
    """configs[2]'s "SATD_8x8 subpel refine" at full resolution, as x264's default preset runs it
    on P slices: refine_subpel (me.c:865-992) at subme 7 (two hpel diamonds of SAD over get_ref
    blocks, the SATD re-score, two qpel SATD diamonds) with b_chroma_me (common/macroblock.c:
    507-509: COST_MV_SATD adds mc_chroma + SATD of U, then V, me.c:833-861) over F 1080p 4:2:0
    pairs of synth.make_subpel_sequence, whose motion is (3.25, 2.5) pixels per frame -- the
    optimum lies at quarter-pel positions, so the diamonds move.  Each partition starts from its
    integer decision: the fused ESA winner of its MB (me_range 16 around mv 0; m->mv = 4 * the
    winner, m->cost its SAD + mv cost, for 8x8 partitions the partition's own SAD there), mv
    limits of analyse.c:336-349.  Legs: 16x16 with chroma ME (refine16_*), 16x16 luma only
    (refine16_luma_*), 8x8 partitions with chroma ME (refine8_*).  VALU fraction on the
    reference's own cmp calls (counted per partition by the kernel, equal to the oracle's count
    in tests/test_gpu_refine*.py): a luma SATD call costs SURVEY §8d's 444 + 192 lane-ops per 64
    pixels, a SAD call 0.75 lane-op slots per pixel (a half-rate v_sad_u8 per 4 absdiffs and a
    v_lerp_u8 per 4 qpel averages), a chroma call the same SATD cost plus 9 lane-ops per pixel
    for mc_chroma's bilinear tap."""
    from x264hip import synth, dist as xd
    W, H = mbw * 16, mbh * 16
    p0, p1 = xd.frame_shard(world * F, world, int(os.environ.get("RANK", "0")))
    luma, stride, origin, nv, cs, co = synth.make_subpel_sequence(p1 - p0 + 1, W, H, 8, start=p0)
    dev = torch.from_numpy(luma).cuda()
    nvd = torch.from_numpy(nv).cuda()
    fstride = luma[0].size
    del luma, nv
    me_range = 16
    par, init, cm, span = tesa_params(mbw, mbh, F, me_range, centre=(0, 0))
    cm_d = torch.from_numpy(cm.view(np.int16)).cuda()
    esa = torch.empty((F * mbw * mbh, 3), dtype=torch.int32, device="cuda")
    x.me_search_esa(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, me_range, me_range,
                    torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(), (cm_d, span), out=esa,
                    fenc_frame_stride=fstride, ref_frame_stride=fstride)
    hv = x.hpel_filter(dev[:-1], origin, stride, W, H)
    planes = [dev[:-1]] + list(hv)
    ext = x.refine_ext(1, 1, 0, fenc_chroma=[nvd[1:]], fenc_chroma_origin=co, fenc_chroma_stride=cs,
                       ref_chroma=[nvd[:-1]], ref_chroma_origin=co, ref_chroma_stride=cs)
    n1 = F * mbw * mbh
    mb = np.arange(n1) % (mbw * mbh)
    emv = esa[:, 1:3].cpu().numpy().astype(np.int64)
    res = {"refine_workload": "1080p 4:2:0 make_subpel_sequence, motion (3.25, 2.5) px/frame, subme 7, "
                              "b_chroma_me on (refine16_luma_*: off), starts at the fused-ESA winners"}
    for leg, i_pixel, chroma in (("refine16", 0, True), ("refine16_luma", 0, False), ("refine8", 3, True)):
        parts = rc_parts = [(0, 0)] if i_pixel == 0 else [(0, 0), (8, 0), (0, 8), (8, 8)]
        k = len(parts)
        n = n1 * k
        j = np.repeat(np.arange(n1), k)
        ox = np.tile([p[0] for p in rc_parts], n1)
        oy = np.tile([p[1] for p in rc_parts], n1)
        mbx, mby = mb[j] % mbw, mb[j] // mbw
        pos = np.stack([j // (mbw * mbh), 16 * mbx + ox, 16 * mby + oy], 1).astype(np.int32)
        rpar = np.zeros((n, 8), np.int16)
        rpar[:, 0], rpar[:, 1] = 4 * emv[j, 0], 4 * emv[j, 1]
        rpar[:, 4], rpar[:, 5] = 4 * (-16 * mbx - 24), 4 * (-16 * mby - 24)
        rpar[:, 6], rpar[:, 7] = 4 * (16 * (mbw - 1 - mbx) + 24), 4 * (16 * (mbh - 1 - mby) + 24)
        if i_pixel == 0:
            init_d = esa[:, 0].contiguous()
        else:                                       # the partition's SAD at the winner + its mv cost
            fo = torch.from_numpy(((pos[:, 0] + 1) * fstride + origin + pos[:, 2] * stride + pos[:, 1])
                                  .astype(np.int64)).cuda()
            ro = torch.from_numpy((pos[:, 0] * fstride + origin + (pos[:, 2] + emv[j, 1]) * stride + pos[:, 1]
                                   + emv[j, 0]).astype(np.int64)).cuda()
            sad = x.pixel_cmp_batch(0, i_pixel, dev, stride, dev, stride, fo, ro)
            mvc = cm[span + 4 * emv[j, 0]].astype(np.int64) + cm[span + 4 * emv[j, 1]]
            init_d = (sad + torch.from_numpy(mvc.astype(np.int32)).cuda()).int().contiguous()
        rpar_d = torch.from_numpy(rpar).cuda()
        pos_d = torch.from_numpy(pos).cuda()
        out = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        ne = torch.empty(n, dtype=torch.int32, device="cuda")

        def step(i_pixel=i_pixel, pos_d=pos_d, rpar_d=rpar_d, init_d=init_d, out=out, ne=ne, chroma=chroma):
            x.me_refine_subpel(dev[1:], origin, stride, planes, origin, stride, i_pixel, 7, pos_d, rpar_d, init_d,
                               (cm_d, span), out=out, fenc_frame_stride=fstride, ref_frame_stride=fstride,
                               nevals=ne, ext=ext if chroma else None)
        wall, ev_ms = timed(step, a.steps, a.warmup, world, graph=True)
        nsad = int((ne & 0xFFFF).sum().item())
        nsatd = int(((ne >> 16) & 0xFF).sum().item())
        nchroma = int((ne >> 24).sum().item())
        px = 256 if i_pixel == 0 else 64
        work = nsad * px * 0.75 + nsatd * px * (444 + 192) / 64 + nchroma * (px // 4) * ((444 + 192) / 64 + 9)
        moved = (out[:, 1:3] != rpar_d[:, 0:2].int()).any(1).float().mean().item()
        qpel = ((out[:, 1:3] & 1) != 0).any(1).float().mean().item()
        res.update({leg + "_partitions_per_s": world * a.steps * n / wall, leg + "_launch_ms": ev_ms,
                    leg + "_partitions_per_launch": n, leg + "_sad_calls_per_part": nsad / n,
                    leg + "_satd_calls_per_part": nsatd / n, leg + "_chroma_calls_per_part": nchroma / n,
                    leg + "_moved_frac": moved, leg + "_qpel_frac": qpel,
                    leg + "_valu_frac": work / (ev_ms * 1e-3) / VALU_LANE_OPS})
    res.update(rates_search(x, a, world, mbw, mbh, F, dev, stride, origin, fstride, planes, ext, cm, cm_d, span))
    res.update(rates_search_ref3(x, a, world, mbw, mbh, F, dev, stride, origin, fstride, planes, (nvd, co, cs), cm_d,
                                 span))
    # planes hold frames 0 .. F-1 (the references of rates_refine's pairs); list 1 of B frame k+1
    # is frame k+2 <= F-1
    res.update(rates_bidir(x, a, world, mbw, mbh, F - 1, dev, stride, origin, fstride, planes, cm_d, span))
    del hv, planes, dev, nvd
    return res


def search_params(mbw, mbh, F, i_pixel, seed=7, motion=(13, 10)):
    """x264_me_search_ref inputs per partition of F frames (x264hip_*_me_search_ref's par / mvc):
    mv limits of analyse.c:330-349 (mv_limit_fpel with the 6-pixel fpel border); a synthetic
    predictor -- x264's mvp and mvc come from the already-coded neighbours (common/mvpred.c), which a
    frame-batched search does not have, so mvp = the true motion +- 8 qpel and four candidates
    (two near the motion, one at zero, one far) stand in for them."""
    rs = np.random.default_rng(seed)
    q = [(0, 0), (8, 0), (0, 8), (8, 8)]
    parts = {0: [(0, 0)], 3: q, 4: [(x, y + d) for x, y in q for d in (0, 4)],
             6: [(x + dx, y + dy) for x, y in q for dy in (0, 4) for dx in (0, 4)]}[i_pixel]
    n1 = F * mbw * mbh
    mb = np.repeat(np.arange(n1), len(parts))
    n = len(mb)
    mbx, mby = (mb % (mbw * mbh)) % mbw, (mb % (mbw * mbh)) // mbw
    pos = np.stack([mb // (mbw * mbh), 16 * mbx + np.tile([p[0] for p in parts], n1),
                    16 * mby + np.tile([p[1] for p in parts], n1)], 1).astype(np.int32)
    par = np.zeros((n, 12), np.int16)
    par[:, 0] = motion[0] + rs.integers(-8, 9, n)
    par[:, 1] = motion[1] + rs.integers(-8, 9, n)
    par[:, 6], par[:, 7] = 4 * (-16 * mbx - 24), 4 * (-16 * mby - 24)
    par[:, 8], par[:, 9] = 4 * (16 * (mbw - 1 - mbx) + 24), 4 * (16 * (mbh - 1 - mby) + 24)
    par[:, 2], par[:, 3] = (par[:, 6] >> 2) + 6, (par[:, 7] >> 2) + 6
    par[:, 4], par[:, 5] = (par[:, 8] >> 2) - 6, (par[:, 9] >> 2) - 6
    par[:, 10] = 4
    mvc = np.zeros((n, 14, 2), np.int16)
    mvc[:, 0, 0], mvc[:, 0, 1] = motion[0] + rs.integers(-6, 7, n), motion[1] + rs.integers(-6, 7, n)
    mvc[:, 1, 0], mvc[:, 1, 1] = motion[0] + rs.integers(-16, 17, n), motion[1] + rs.integers(-16, 17, n)
    mvc[:, 3, 0], mvc[:, 3, 1] = rs.integers(-120, 121, n), rs.integers(-80, 81, n)
    return pos, par, mvc


def rates_search(x, a, world, mbw, mbh, F, dev, stride, origin, fstride, planes, ext, cm, cm_d, span):
    """x264_me_search_ref at full resolution (x264hip_*_me_search_ref: predictors, integer search,
    refine_subpel with chroma ME) as x264's default preset runs it on P slices -- HEX, subme 7,
    me_range 16 (common/base.c:439-441) -- over every 16x16 MB (search16_hex_*) and every 8x8
    partition (search8_hex_*) of the F pairs of rates_refine's quarter-pel sequence, and UMH
    (--me umh, the slower presets) on 16x16 (search16_umh_*), every 4x4 partition (search4_hex_*:
    --partitions p4x4, analyse.c:1685-1760) and the exhaustive ESA window (search16_esa_*: --me
    esa, me.c:618-631), and the 16x16 HEX search with x264's own predictors over each frame's MB
    wavefront (search16_hex_wavefront_*, me_analyse_p16x16).  Rates in partitions/s; the
    candidates the reference evaluates (its fpelcmp / get_ref / refine calls, counted by the
    kernels) give the absdiff rate against the v_sad_u8 peak."""
    res = {"search_workload": "rates_refine's sequence, synthetic mvp / mvc (search_params), subme 7, me_range 16, "
                              "b_chroma_me on, the whole x264_me_search_ref per launch"}
    for leg, i_pixel, me in (("search16_hex", 0, 1), ("search16_umh", 0, 2), ("search8_hex", 3, 1),
                             ("search4_hex", 6, 1), ("search16_esa", 0, 3)):
        pos, par, mvc = search_params(mbw, mbh, F, i_pixel)
        n = len(pos)
        pos_d, par_d, mvc_d = (torch.from_numpy(v).cuda() for v in (pos, par, mvc))
        out = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        ne = torch.empty((n, 2), dtype=torch.int32, device="cuda")

        def step(i_pixel=i_pixel, me=me, pos_d=pos_d, par_d=par_d, mvc_d=mvc_d, out=out, ne=ne):
            x.me_search_ref(dev[1:], origin, stride, dev[:-1], planes, origin, stride, i_pixel, me, 7, 16, pos_d,
                            par_d, mvc_d, (cm_d, span), out=out, fenc_frame_stride=fstride,
                            ref_frame_stride=fstride, nevals=ne, ext=ext)
        wall, ev_ms = timed(step, a.steps, a.warmup, world, graph=True)
        nf = int((ne[:, 0] & 0xFFFF).sum().item())
        nh = int((ne[:, 0] >> 16).sum().item())
        rsad = int((ne[:, 1] & 0xFFFF).sum().item())
        rsatd = int(((ne[:, 1] >> 16) & 0xFF).sum().item())
        rchroma = int((ne[:, 1] >> 24).sum().item())
        px = {0: 256, 3: 64, 4: 32, 6: 16}[i_pixel]
        cands = nf + nh + rsad + rsatd
        res.update({leg + "_partitions_per_s": world * a.steps * n / wall, leg + "_launch_ms": ev_ms,
                    leg + "_partitions_per_launch": n, leg + "_fpel_calls_per_part": nf / n,
                    leg + "_hpel_calls_per_part": nh / n, leg + "_refine_sad_per_part": rsad / n,
                    leg + "_refine_satd_per_part": rsatd / n, leg + "_refine_chroma_per_part": rchroma / n,
                    leg + "_candidates_per_s": world * a.steps * cands / wall,
                    leg + "_absdiff_frac": cands * px / (ev_ms * 1e-3) / SAD_PEAK_ABSDIFF,
                    leg + "_mv_found_frac": ((out[:, 1] == 13) & (out[:, 2] == 10)).float().mean().item()})
    # the same 16x16 HEX search with x264's own predictors (me_analyse_p16x16: mvp / mvc from the
    # frame's decided neighbours, mvpred.c:129-157, 519-600, i_mv_range 512) -- the raster
    # dependency as a wavefront of MB anti-diagonals, one predictor + one search launch each
    n = F * mbw * mbh
    out = torch.empty((F, mbw * mbh, 4), dtype=torch.int32, device="cuda")
    ne = torch.empty((F, mbw * mbh, 2), dtype=torch.int32, device="cuda")

    def wstep():
        x.me_analyse_p16x16(dev[1:], origin, stride, dev[:-1], planes, origin, stride, mbw, mbh, F, 1, 7, 16,
                            (cm_d, span), mv_range=512, out=out, nevals=ne, ext=ext, fenc_frame_stride=fstride,
                            ref_frame_stride=fstride)
    # (eager, fewer steps: ~510 launches a step would make a graph of tens of thousands of
    # nodes, and the step is long enough to keep the queue fed)
    ws = min(a.steps, 10)
    wall, ev_ms = timed(wstep, ws, min(a.warmup, 2), world)
    nf = int((ne[..., 0] & 0xFFFF).sum().item())
    res.update({"search16_hex_wavefront_mbs_per_s": world * ws * n / wall,
                "search16_hex_wavefront_step_ms": ev_ms, "search16_hex_wavefront_diagonals": mbw + 2 * (mbh - 1),
                "search16_hex_wavefront_fpel_calls_per_part": nf / n,
                "search16_hex_wavefront_mv_found_frac":
                    ((out[..., 1] == 13) & (out[..., 2] == 10)).float().mean().item()})
    return res


def rates_bidir(x, a, world, mbw, mbh, F, dev, stride, origin, fstride, planes, cm_d, span):
    """x264_me_refine_bidir_satd (me.c:994-1183) over every 16x16 MB (bidir16_*) and every 8x8
    partition (bidir8_*) of F B frames of rates_refine's quarter-pel sequence: frame k+1 between
    list 0 = frame k and list 1 = frame k+2 (true motion +(13, 10) and -(13, 10) qpel), starting
    from the true mvs +- 4 qpel (the list searches' winners stand-in), mvps +- 8, i_weight 32
    (the default without weighted bipred) on half the partitions and 24 on the rest, SATD mbcmp.
    Rates in partitions/s; the pairs the reference scores (mbcmp calls counted by the kernel)
    give the absdiff-equivalent work."""
    if F < 2:
        return {}
    Fb = F - 1
    res = {"bidir_workload": "rates_refine's sequence, B frame k+1 between frames k and k+2, starts true mv +- 4 "
                             "qpel, i_weight 32 / 24, SATD"}
    for leg, i_pixel in (("bidir16", 0), ("bidir8", 3)):
        pos, par, _ = search_params(mbw, mbh, Fb, i_pixel, seed=11)
        n = len(pos)
        rs = np.random.default_rng(12)
        bp = np.zeros((n, 12), np.int16)
        bp[:, 0], bp[:, 1] = 13 + rs.integers(-4, 5, n), 10 + rs.integers(-4, 5, n)
        bp[:, 2], bp[:, 3] = -13 + rs.integers(-4, 5, n), -10 + rs.integers(-4, 5, n)
        bp[:, 4], bp[:, 5] = 13 + rs.integers(-8, 9, n), 10 + rs.integers(-8, 9, n)
        bp[:, 6], bp[:, 7] = -13 + rs.integers(-8, 9, n), -10 + rs.integers(-8, 9, n)
        bp[:, 8:12] = par[:, 6:10]
        wt = np.where(rs.random(n) < 0.5, 32, 24).astype(np.int32)
        pos_d, bp_d, wt_d = (torch.from_numpy(v).cuda() for v in (pos, bp, wt))
        out = torch.empty((n, 4), dtype=torch.int32, device="cuda")
        ne = torch.empty(n, dtype=torch.int32, device="cuda")
        l0 = [pl[0:Fb] for pl in planes]
        l1 = [pl[2:Fb + 2] for pl in planes]

        def step(i_pixel=i_pixel, pos_d=pos_d, bp_d=bp_d, wt_d=wt_d, out=out, ne=ne, l0=l0, l1=l1):
            x.me_refine_bidir(dev[1:Fb + 1], origin, stride, l0, l1, origin, stride, i_pixel, pos_d, bp_d, wt_d,
                              (cm_d, span), out=out, nevals=ne, fenc_frame_stride=fstride, ref_frame_stride=fstride)
        wall, ev_ms = timed(step, a.steps, a.warmup, world, graph=True)
        calls = int((ne & 0xFFFF).sum().item())
        passes = int((ne >> 16).sum().item())
        px = 256 if i_pixel == 0 else 64
        res.update({leg + "_partitions_per_s": world * a.steps * n / wall, leg + "_launch_ms": ev_ms,
                    leg + "_partitions_per_launch": n, leg + "_calls_per_part": calls / n,
                    leg + "_passes_per_part": passes / n,
                    leg + "_pairs_per_s": world * a.steps * calls / wall,
                    leg + "_found_frac": ((out[:, 0] == 13) & (out[:, 1] == 10) & (out[:, 2] == -13) &
                                          (out[:, 3] == -10)).float().mean().item()})
    return res


def rates_search_ref3(x, a, world, mbw, mbh, F, dev, stride, origin, fstride, planes, chroma, cm_d, span):
    """x264's default P16x16 search over three references (ref = 3, common/base.c:384, with
    b_early_terminate, analyse.c:303): mb_analyse_inter_p16x16's loop (analyse.c:1260-1314) as one
    x264hip_*_me_search_ref_thresh launch per reference, every MB's p_halfpel_thresh chained
    through them (me.c:931-944) with the i_ref_cost adjustments (analyse.c:1271, 1310).  Frames
    3..F of rates_refine's sequence search references 1, 2 and 3 frames back (true motion 1x, 2x,
    3x the per-frame (13, 10) qpel; synthetic predictors around it, search_params); i_ref_cost =
    lambda * te() bits of ref 0 / 1 / 2 at num_ref_idx 3 (1, 3, 3 bits, lambda 12 -- qp 26's
    x264_lambda_tab).  Rates: MB-reference searches/s (search16_hex_ref3_partitions_per_s) and
    MBs/s (all three references), the fraction of later-reference searches the exit ended."""
    if F < 3:
        return {}
    Fr = F - 2
    n = Fr * mbw * mbh
    INT_MAX = (1 << 31) - 1
    thr = torch.full((n,), INT_MAX, dtype=torch.int32, device="cuda")
    legs = []
    for k in range(3):
        pos, par, mvc = search_params(mbw, mbh, Fr, 0, seed=7 + k, motion=(13 * (k + 1), 10 * (k + 1)))
        rf = slice(2 - k, F - k)                    # reference k + 1 frames back (planes: frames 0 .. F-1)
        nvd, co, cs = chroma
        ek = x.refine_ext(1, 1, 0, fenc_chroma=[nvd[3:]], fenc_chroma_origin=co, fenc_chroma_stride=cs,
                          ref_chroma=[nvd[rf]], ref_chroma_origin=co, ref_chroma_stride=cs)
        legs.append(dict(pos=torch.from_numpy(pos).cuda(), par=torch.from_numpy(par).cuda(),
                         mvc=torch.from_numpy(mvc).cuda(), planes=[p[rf] for p in planes], ext=ek,
                         rcost=torch.full((n,), 12 * (1 if k == 0 else 3), dtype=torch.int32, device="cuda"),
                         out=torch.full((n, 4), -7, dtype=torch.int32, device="cuda"),
                         ne=torch.empty((n, 2), dtype=torch.int32, device="cuda")))

    def step():
        thr.fill_(INT_MAX)
        for L in legs:
            x.me_search_ref(dev[3:], origin, stride, L["planes"][0], L["planes"], origin, stride, 0, 1, 7, 16, L["pos"],
                            L["par"], L["mvc"], (cm_d, span), out=L["out"], fenc_frame_stride=fstride,
                            ref_frame_stride=fstride, nevals=L["ne"], ext=L["ext"], halfpel_thresh=thr,
                            ref_cost=L["rcost"])
    wall, ev_ms = timed(step, a.steps, a.warmup, world, graph=True)
    for L in legs:                                  # the last step's outputs: mark the early exits
        L["out"][:, 3].fill_(-7)
    step()
    torch.cuda.synchronize()
    early = [int((L["out"][:, 3] == -7).sum().item()) for L in legs]
    qcalls = [int(((L["ne"][:, 1] >> 16) & 0xFF).sum().item()) for L in legs]
    return {"search16_hex_ref3_partitions_per_s": world * a.steps * 3 * n / wall,
            "search16_hex_ref3_mbs_per_s": world * a.steps * n / wall,
            "search16_hex_ref3_step_ms": ev_ms, "search16_hex_ref3_mbs_per_step": n,
            "search16_hex_ref3_early_exit_frac": [e / n for e in early],
            "search16_hex_ref3_refine_satd_per_part": [q / n for q in qcalls],
            "search16_hex_ref3_workload": "frames 3..F of rates_refine's sequence, references 1 / 2 / 3 frames "
                                          "back, HEX subme 7 me_range 16 chroma ME, i_ref_cost 12 / 36 / 36, "
                                          "one launch per reference, p_halfpel_thresh chained"}


def rates_full8(x, a, world, dev, origin, stride, fstride, mbw, mbh, F, bd=8):
    """8x8 quadrant tables (me_search_full8, the lookup mode's source for PIXEL_16x8 / 8x16 /
    8x8, analyse.c:1425,1480,1546) over the F pairs at range R: the VALU fraction (256
    absdiffs per 16x16 candidate, the same work as the 16x16 table) and the HBM fraction of
    the four quadrant tables written (8 B per candidate at the padded pitch) plus the planes."""
    R = a.range
    w, pitch = 2 * R + 1, x.me_table_pitch(R)
    t8 = torch.empty((F, mbh, mbw, 4, w, pitch), dtype=torch.int16, device="cuda")

    def step():
        x.me_search_full8(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, R, table8=t8,
                          fenc_frame_stride=fstride, ref_frame_stride=fstride)
    wall, ev_ms = timed(step, a.steps, a.warmup, world)
    cands = F * mbw * mbh * w * w
    pre = "full8" if bd == 8 else "full8_10"
    peak = SAD_PEAK_ABSDIFF if bd == 8 else SAD_PEAK_ABSDIFF / 2
    es = dev.element_size()
    moved = t8.numel() * 2 + 2 * F * (mbh * 16 + 64) * stride * es
    res = {pre + "_candidates_per_s": world * a.steps * cands / wall, pre + "_launch_ms": ev_ms,
           pre + "_valu_frac": cands * 256 / (ev_ms * 1e-3) / peak,
           pre + "_hbm_frac": moved / (ev_ms * 1e-3) / HBM_PEAK, pre + "_table_bytes": t8.numel() * 2}
    del t8
    return res


def rates_esa8(x, a, world, dev, origin, stride, fstride, mbw, mbh, F, pre="esa8"):
    """ESA decisions of every MB's eight sub-partitions (me_search_esa8: PIXEL_16x8 x2, 8x16 x2,
    8x8 x4, me.c:618-631 per partition, analyse.c:1425,1480,1546) over the F pairs at me_range
    16, template radius 16 around each MB's centre (mv 0).  Two contents: every partition's
    window centred on its MB's (the shared-absdiff pass decides all of them), and a quarter of
    the partitions starting from a predictor up to 3 pixels off it (x264 starts each partition
    from its own best predictor; those windows' outside strips take the direct pass); and the
    first with every centre at x = 1 (template rows off the dword grid).  The
    fraction is taken on the shared work, 256 byte absdiffs per 16x16 window candidate (the
    quadrant-table search's basis, full8_valu_frac); the first content is checked against the
    direct pass alone (range 0)."""
    me_range = R = a.range
    n1 = mbw * mbh
    par1, init1, cm, span = tesa_params(mbw, mbh, F, me_range, centre=(0, 0))
    par = np.repeat(par1, 8, axis=0)
    init = np.repeat(init1, 8)
    cm_d = torch.from_numpy(cm.view(np.int16)).cuda()
    cen_d = torch.zeros((F * n1, 2), dtype=torch.int16, device="cuda")
    rs = np.random.default_rng(17)
    par_s = par.copy()
    move = rs.random(len(par)) < 0.25
    off = rs.integers(-3, 4, (len(par), 2))
    par_s[:, 0] += np.where(move, off[:, 0], 0).astype(np.int16)
    par_s[:, 1] += np.where(move, off[:, 1], 0).astype(np.int16)
    par_s[:, 2], par_s[:, 3] = 4 * par_s[:, 0], 4 * par_s[:, 1]
    # a centre off the dword grid (x = 1): the template's row loads are misaligned
    par_o = np.repeat(tesa_params(mbw, mbh, F, me_range, centre=(1, 0))[0], 8, axis=0)
    cen_o = torch.tensor([1, 0], dtype=torch.int16, device="cuda").repeat(F * n1, 1)
    out = torch.empty((len(par), 3), dtype=torch.int32, device="cuda")
    init_d = torch.from_numpy(init).cuda()
    res = {}
    for tag, pp, cc in ((pre, par, cen_d), (pre + "_spread", par_s, cen_d), (pre + "_offgrid", par_o, cen_o)):
        par_d = torch.from_numpy(pp).cuda()

        def step(par_d=par_d, cc=cc):
            x.me_search_esa8(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, R, me_range, cc,
                             par_d, init_d, (cm_d, span), out=out, fenc_frame_stride=fstride,
                             ref_frame_stride=fstride)
        wall, ev_ms = timed(step, a.steps, a.warmup, world)
        cands = esa_window_candidates(par1, me_range)        # 16x16 windows: the shared absdiffs
        res[tag + "_step_ms"] = ev_ms
        res[tag + "_partitions_per_s"] = world * a.steps * len(pp) / wall
        # (10 bit: v_sad_u16 folds two absdiffs where v_sad_u8 folds four)
        res[tag + "_frac"] = cands * 256 / (ev_ms * 1e-3) / (SAD_PEAK_ABSDIFF / (2 if pre == "esa8_10" else 1))
        if tag == pre:
            direct = x.me_search_esa8(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, 0, me_range,
                                      cen_d, par_d, init_d, (cm_d, span), fenc_frame_stride=fstride,
                                      ref_frame_stride=fstride)
            if not torch.equal(out, direct):
                raise SystemExit("bench: me_search_esa8 template and direct passes disagree")
        elif tag == pre + "_spread":
            res[tag + "_moved_fraction"] = float(move.mean())
    return res


def rates_ssd(x, a, world, dev, origin, stride, F):
    """plane SSD (x264_pixel_ssd_wxh, the per-frame PSNR sum of encoder.c:2499) over the F
    1080p pairs: frames/s and the fraction of HBM (two w x h planes read)."""
    out = torch.empty(F, dtype=torch.int64, device="cuda")
    # the reconstructed planes as a buffer of their own (in an encoder fenc and fdec are
    # different frames): with both operands slices of one sequence, frame f+1 is read as the
    # source of pair f+1 and the reference of pair f, and the second read comes from cache
    recon = dev[:-1].clone()

    def step():
        x.ssd_plane_batch(dev[1:], origin, stride, recon, origin, stride, a.width, a.height, F, out=out)
    wall, ev_ms = timed(step, a.steps, a.warmup, world, graph=True)
    return {"ssd_plane_frames_per_s": world * a.steps * F / wall, "ssd_plane_launch_ms": ev_ms,
            "ssd_plane_hbm_frac": F * 2 * a.width * a.height / (ev_ms * 1e-3) / HBM_PEAK}


def rates_10bit(x, a, world, mbw, mbh, F):
    """configs[4] side rates: 10-bit full search (v_sad_u16 path) over F frame pairs and
    10-bit fused 8x8 DCT + quant_8x8 (int32 coefficients) over --tframes pairs of the
    same motion."""
    from x264hip import synth, dist as xd
    R = a.range
    p0, p1 = xd.frame_shard(world * F, world, int(os.environ.get("RANK", "0")))
    planes, stride, origin = synth.make_sequence(p1 - p0 + 1, mbw * 16, mbh * 16, 10, start=p0)
    dev = torch.from_numpy(planes.view(np.int16)).cuda()
    fstride = planes[0].size
    table = torch.empty((F, mbh, mbw, 2 * R + 1, x.me_table_pitch(R)), dtype=torch.int32, device="cuda")

    def mstep():
        x.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, R, table=table,
                         fenc_frame_stride=fstride, ref_frame_stride=fstride)
    wall, ev_ms = timed(mstep, a.steps, a.warmup, world)
    cands = F * mbw * mbh * (2 * R + 1) ** 2
    res = {"me10_candidates_per_s": world * a.steps * cands / wall, "me10_launch_ms": ev_ms,
           "me10_absdiff_frac_of_v_sad_u16_peak": cands * 256 / (ev_ms * 1e-3) / VALU_LANE_OPS}
    del table
    res.update(rates_full8(x, a, world, dev, origin, stride, fstride, mbw, mbh, F, bd=10))
    res.update(rates_esa8(x, a, world, dev, origin, stride, fstride, mbw, mbh, F, pre="esa8_10"))
    del dev
    flat = [16] * 64
    _, _, q8m, q8b = x.cqm_init(10, [flat] * 8)
    mf8 = torch.from_numpy(q8m[1, 26 + 12].copy()).cuda()
    bs8 = torch.from_numpy(q8b[1, 26 + 12].copy()).cuda()
    TF = a.tframes                                  # >= 64 frames per transform launch
    t0, t1 = xd.frame_shard(world * TF, world, int(os.environ.get("RANK", "0")))
    tplanes, _, _ = synth.make_sequence(t1 - t0 + 1, mbw * 16, mbh * 16, 10, start=t0)
    dev = torch.from_numpy(tplanes.view(np.int16)).cuda()
    del tplanes
    nmb = TF * mbw * mbh
    dct = torch.empty((nmb, 256), dtype=torch.int32, device="cuda")
    nz = torch.empty(nmb, dtype=torch.int32, device="cuda")
    pred = dev[:-1].clone()                         # a buffer of its own, as in the 8-bit legs

    def dstep():
        x.mb_dct_quant(8, dev[1:], origin, stride, pred, origin, stride, mbw, mbh, TF, mf8, bs8, dct=dct,
                       nz=nz, fenc_frame_stride=fstride, pred_frame_stride=fstride)
    wall, ev_ms = timed(dstep, a.steps, a.warmup, world)
    blocks = nmb * 4
    res["dct8_quant10_blocks_per_s"] = world * a.steps * blocks / wall
    res["dct8_quant10_hbm_frac"] = blocks * (128 + 128 + 256) / (ev_ms * 1e-3) / HBM_PEAK
    res["dct8_quant10_launch_ms"] = ev_ms
    return res


def rates_2160p(x, a, world):
    """configs[3] per GPU (frame-per-GPU across the node): 2160p, full search range 16
    + fused 4x4 DCT+quant of each new frame against its predecessor.  Two rates:
    frames resident in HBM, and the streaming form where every new frame is uploaded
    from pinned host memory (the reference frame is the previous upload, already on
    the device) on a copy stream overlapped with the previous frame's kernels."""
    from x264hip import synth, dist as xd
    W, H, R = 3840, 2160, a.range                     # 240 x 135 MBs (2160 = 135 * 16, no MB padding)
    mbw, mbh = W // 16, H // 16
    nf = 8
    p0, _ = xd.frame_shard(world * nf, world, int(os.environ.get("RANK", "0")))
    planes, stride, origin = synth.make_sequence(nf + 1, W, H, 8, start=p0)
    fsz = planes[0].size
    host = torch.from_numpy(planes).pin_memory()
    ring = torch.empty((3,) + planes.shape[1:], dtype=torch.uint8, device="cuda")
    table = torch.empty((1, mbh, mbw, 2 * R + 1, x.me_table_pitch(R)), dtype=torch.int16, device="cuda")
    flat = [16] * 64
    q4m, q4b, _, _ = x.cqm_init(8, [flat] * 8)
    mf4 = torch.from_numpy(q4m[1, 26].copy()).cuda()
    bs4 = torch.from_numpy(q4b[1, 26].copy()).cuda()
    dct = torch.empty((mbw * mbh, 256), dtype=torch.int16, device="cuda")
    nz = torch.empty(mbw * mbh, dtype=torch.int32, device="cuda")
    dev_all = host.cuda()
    cand = mbw * mbh * (2 * R + 1) ** 2

    def work(cur, ref, c_fs=fsz, r_fs=fsz):
        x.me_search_full(cur, origin, stride, ref, origin, stride, mbw, mbh, 1, R, table=table,
                         fenc_frame_stride=c_fs, ref_frame_stride=r_fs)
        x.mb_dct_quant(4, cur, origin, stride, ref, origin, stride, mbw, mbh, 1, mf4, bs4, dct=dct, nz=nz,
                       fenc_frame_stride=c_fs, pred_frame_stride=r_fs)

    k = [0]

    def resident():
        i = k[0] % nf
        work(dev_all[i + 1:i + 2], dev_all[i:i + 1])
        k[0] += 1
    wall, ev_ms = timed(resident, a.steps, min(a.warmup, 50), world)
    res = {"2160p_resident_candidates_per_s": world * a.steps * cand / wall,
           "2160p_resident_frame_ms": wall / a.steps * 1e3}
    # sdma: the runtime's copy engine on a plain side stream; kernel: x264hip_upload on the
    # copy stream of a CU-partitioned pair (x264hip_stream_pair_create: 16 CUs for the copy,
    # the other 240 for the search), so the upload's workgroups never wait for CU slots
    normal = (torch.cuda.current_stream(), torch.cuda.Stream())
    split = x.stream_pair(16)
    done = [torch.cuda.Event() for _ in range(3)]
    ready = [torch.cuda.Event() for _ in range(3)]
    state = {"n": 0, "how": "sdma", "streams": normal}

    def streaming():
        n = state["n"]
        comp, copy = state["streams"]
        cur, ref = (n + 1) % 3, n % 3
        with torch.cuda.stream(copy):                 # upload frame n+1 while frame n-1's kernels may still run
            copy.wait_event(done[cur])
            if state["how"] == "sdma":                # the runtime's copy engine
                ring[cur].copy_(host[(n + 1) % (nf + 1)], non_blocking=True)
            else:                                     # x264hip_upload: a kernel reading the pinned pages
                x.upload(ring[cur], host[(n + 1) % (nf + 1)])
            ready[cur].record(copy)
        with torch.cuda.stream(comp):
            comp.wait_event(ready[cur])
            comp.wait_event(ready[ref])
            work(ring[cur:cur + 1], ring[ref:ref + 1], c_fs=0, r_fs=0)
            done[ref].record(comp)
        state["n"] = n + 1

    def upload_only():
        x.upload(ring[1], host[1])
    # The host link is shared with the node's other GPUs and swings between runs (the same
    # leg read 0.18-0.25 ms per frame within one process, profiles/r03e_*): the link alone
    # and the two streaming forms are timed in interleaved rounds and each reported as the
    # median round, so their ratio compares like with like.
    rounds = {"upload": [], "sdma": [], "kernel": []}
    for _ in range(5):
        wall, _ = timed(upload_only, a.steps, min(a.warmup, 50), world)
        rounds["upload"].append(wall / a.steps * 1e3)
        for how, streams in (("sdma", normal), ("kernel", split)):
            torch.cuda.synchronize()
            state.update(n=0, how=how, streams=streams)
            ring[0].copy_(host[0])
            ready[0].record()
            for ev in done:
                ev.record()
            wall, _ = timed(streaming, a.steps, min(a.warmup, 50), world)
            torch.cuda.synchronize()
            rounds[how].append(wall / a.steps * 1e3)
    med = {k: float(np.median(v)) for k, v in rounds.items()}
    res["2160p_upload_only_ms"] = med["upload"]
    res["2160p_upload_only_GBps"] = fsz / (med["upload"] * 1e-3) / 1e9
    res["2160p_stream_rounds_ms"] = {k: [round(t, 4) for t in v] for k, v in rounds.items()}
    for how in ("sdma", "kernel"):
        res[f"2160p_pcie_{how}_candidates_per_s"] = world * cand / (med[how] * 1e-3)
        res[f"2160p_pcie_{how}_frame_ms"] = med[how]
    # host time to enqueue one frame (no GPU wait inside streaming()): a leg whose host side
    # were slower than its GPU side would measure Python, not the link
    t0 = time.perf_counter()
    for _ in range(a.steps):
        streaming()
    res["2160p_pcie_kernel_host_enqueue_ms"] = (time.perf_counter() - t0) / a.steps * 1e3
    torch.cuda.synchronize()
    x.stream_pair_destroy(split)
    best = max(("sdma", "kernel"), key=lambda h: res[f"2160p_pcie_{h}_candidates_per_s"])
    res["2160p_pcie_inclusive_candidates_per_s"] = res[f"2160p_pcie_{best}_candidates_per_s"]
    res["2160p_pcie_inclusive_frame_ms"] = res[f"2160p_pcie_{best}_frame_ms"]
    res["2160p_pcie_inclusive_upload"] = best
    res["2160p_upload_bytes_per_frame"] = int(fsz)
    res["2160p_pcie_inclusive_vs_upload_only"] = res["2160p_pcie_inclusive_frame_ms"] / res["2160p_upload_only_ms"]
    del dev_all, ring, table, host
    return res


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_lookahead(orc, planes, origin, stride, mbw, mbh, nthr, bounded):
    """CPU anchors of the lookahead legs on the same frames: the P search (lowres_inter_cost,
    HEX subme 4) per pair and the B leg (lowres_bidir_cost, both lists searched) per triplet --
    one thread, and nthr threads over independent pairs (ctypes drops the GIL in the oracle) --
    and x264_weights_analyse on the bench's fade of frame 1 (one thread, per call)."""
    from concurrent.futures import ThreadPoolExecutor
    W, H = mbw * 16, mbh * 16
    ls = (W // 2 + 64 + 63) // 64 * 64
    lo = 32 * ls + 32
    nf = min(planes.shape[0], 5)
    lr = [[p.ravel() for p in orc.frame_init_lowres(8, planes[i].ravel(), origin, stride, W, H, ls)] for i in range(nf)]
    ic = [orc.lowres_intra_cost(8, lr[i][0], lo, ls, mbw, mbh, lam=1)[0] for i in range(nf)]
    res = {}

    def p_pair(k):
        return orc.lowres_inter_cost(8, lr[k + 1][0], lr[k], lo, ls, mbw, mbh, ic[k + 1])

    def b_trip(k):
        z = np.zeros((mbw * mbh, 2), np.int16)
        c = np.zeros(mbw * mbh, np.int32)
        return orc.lowres_bidir_cost(8, lr[k + 1][0], lr[k], lr[k + 2], lo, ls, mbw, mbh, 3, z, c, z, c)

    pool = ThreadPoolExecutor(nthr)
    for name, fn, n in (("lowres_me_pairs_per_s", p_pair, nf - 1), ("lowres_bidir_triplets_per_s", b_trip, nf - 2)):
        res[name + "_1t"] = bounded(lambda fn=fn: fn(0) and 1, 1)[0]
        jobs = [k % n for k in range(nthr)]
        res[name] = bounded(lambda fn=fn, jobs=jobs: list(pool.map(fn, jobs)) and 1, len(jobs))[0]
    pool.shutdown()
    # the weight search: frame 1 faded (x 0.85 + 12) against frame 0, as rates_weightp
    fade = np.clip(np.floor(planes[1].astype(np.float64) * 0.85 + 12 + 0.5), 0, 255).astype(np.uint8)
    fl = [p.ravel() for p in orc.frame_init_lowres(8, fade.ravel(), origin, stride, W, H, ls)]
    fic = orc.lowres_intra_cost(8, fl[0], lo, ls, mbw, mbh, lam=1)[0]
    st = [orc.frame_pixel_stats(8, [p.ravel(), None, None], [origin, 0, 0], [stride, 0, 0], mbw, mbh, 0)
          for p in (fade, planes[0])]
    mvs = orc.lowres_inter_cost(8, fl[0], lr[0], lo, ls, mbw, mbh, fic)[0]
    res["pixel_stats_frames_per_s_1t"] = bounded(lambda: orc.frame_pixel_stats(
        8, [fade.ravel(), None, None], [origin, 0, 0], [stride, 0, 0], mbw, mbh, 0) and 1, 1)[0]
    for name, kw in (("la", dict(b_lookahead=True)), ("enc", dict(b_lookahead=False, subme=7, mvs=mvs))):
        rate = bounded(lambda kw=kw: orc.weights_analyse(8, fl[0], lr[0], lo, ls, mbw, mbh, fic, st[0], st[1],
                                                         **kw) and 1, 1)[0]
        res["weightp_%s_ms_1t" % name] = 1e3 / rate
    # SSIM of the 1080p pair as rates_ssim measures it: the whole frame on one thread, and the
    # encoder's 68 bands over the CPU share's threads (ctypes releases the GIL in the oracle)
    res["ssim_frames_per_s_1t"] = bounded(lambda: orc.ssim_wxh(8, planes[1].ravel(), origin + 2, stride,
                                                               planes[0].ravel(), origin + 2, stride, W - 2, H)
                                          and 1, 1)[0]
    import importlib
    bands = importlib.import_module("x264hip").ssim_encoder_bands(mbh, min(H, 1080))
    fa, fb = planes[1].ravel(), planes[0].ravel()
    # one pthread per contiguous run of bands (cpubench.c): a thread-pool task per band cost more
    # than the band's ~17 us of work (round 5 measured 343.6 frames/s on 16 threads this way,
    # below the 1-thread whole-frame rate)
    bl = np.ascontiguousarray(np.asarray(bands)[:, :2], np.int32)
    res["ssim_bands_frames_per_s"] = bounded(lambda: orc.ssim_bands_mt(fa, origin + 2, stride, fb, origin + 2, stride,
                                                                       W - 2, bl, nthr) and 1, 1)[0]
    return res


def cpu_search(orc, mbw, mbh, nthr, bounded):
    """The oracle's x264_me_search_ref (HEX, subme 7, chroma ME: rates_search's search16_hex leg) on
    one pair of rates_refine's quarter-pel sequence, on one thread and on the CPU share's threads
    (a frame's MB rows split over them; ctypes releases the GIL in the oracle)."""
    from concurrent.futures import ThreadPoolExecutor
    from x264hip import synth
    W, H = mbw * 16, mbh * 16
    luma, stride, origin, nv, cs, co = synth.make_subpel_sequence(2, W, H, 8)
    ref, fenc = luma[0].ravel(), luma[1].ravel()
    planes = [ref] + [h.ravel() for h in orc.frame_filter(8, ref, origin, stride, W, H)]
    pos, par, mvc = search_params(mbw, mbh, 1, 0)
    par_c = np.ascontiguousarray(par)
    span = 16384
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    cm = np.minimum((4 * logs + 0.5).astype(np.int64), 65535).astype(np.uint16)
    ext = orc.refine_ext(1, 1)

    def rows(r0, r1):
        sel = slice(r0 * mbw, r1 * mbw)
        return orc.me_search_ref(8, fenc, origin, stride, planes, ref, origin, stride, 0, 1, 7, 16, pos[sel, 1:],
                                 par_c[sel], mvc[sel], cm, span, ext=ext, fenc_c=[nv[1].ravel()], fc_origin=co,
                                 fcs=cs, ref_c=[nv[0].ravel()], rc_origin=co, rcs=cs)
    res = {"search16_hex_partitions_per_s_1t": bounded(lambda: rows(0, 4) and 1, 4 * mbw)[0]}
    pool = ThreadPoolExecutor(nthr)
    cuts = [(mbh * k // nthr, mbh * (k + 1) // nthr) for k in range(nthr)]
    res["search16_hex_partitions_per_s"] = bounded(lambda: list(pool.map(lambda c: rows(*c), cuts)) and 1,
                                                   mbw * mbh)[0]
    pool.shutdown()
    return res


def cpu_baseline(planes, origin, stride, mbw, mbh, R, seconds):
    """The oracle (kind "port": reference C kernels restated, -O3 -march=x86-64-v3) on the
    host cores, each leg time-bounded: the headline full-search tables (value: the box's
    CPU share of threads), and beside it one thread, the fused DCT+quant 4x4 / 8x8 and the
    SATD 8x8 qpel candidates of configs[2] -- every GPU rate of that config gets a CPU
    rate on the same inputs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc  # cpu_baseline leg only
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    nthr = min(16, share)                            # the GPU box's CPU share per GPU is 16
    fenc, ref = planes[1].ravel(), planes[0].ravel()

    def bounded(fn, units):
        """repeat fn() (each call = `units` work units) for `seconds`; units/s, calls, threads"""
        n, used = 0, 1
        t0 = time.perf_counter()
        while True:
            used = fn()
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
        dt = time.perf_counter() - t0
        return n * units / dt, n, used, dt

    res = {}
    cand_per_mb = (2 * R + 1) ** 2
    me_rate, me_calls, me_used, me_dt = bounded(
        lambda: orc.me_search_full_mt(fenc, origin, stride, ref, origin, stride, mbw, mbh, R, nthr)[1],
        mbw * mbh * cand_per_mb)
    # every CPU the process may run on (1 thread and nproc threads); on the GPU
    # box that is the whole host's count, of which the job's cgroup grants a share
    if share > nthr:
        res["all_cpus_candidates_per_s"], _, res["all_cpus_threads"], _ = bounded(
            lambda: orc.me_search_full_mt(fenc, origin, stride, ref, origin, stride, mbw, mbh, R, share)[1],
            mbw * mbh * cand_per_mb)
    else:
        res["all_cpus_candidates_per_s"], res["all_cpus_threads"] = me_rate, me_used
    band = 4                                          # one thread: 4 MB rows per call keeps the leg bounded
    res["single_thread_candidates_per_s"] = bounded(
        lambda: orc.me_search_full_mt(fenc, origin, stride, ref, origin, stride, mbw, band, R, 1)[1],
        mbw * band * cand_per_mb)[0]
    flat = [16] * 64
    q4m, q4b, q8m, q8b = orc.cqm_init(8, [flat] * 8)
    for t, mf, bs in ((4, q4m[1, 26], q4b[1, 26]), (8, q8m[1, 26], q8b[1, 26])):
        blocks = mbw * mbh * (16 if t == 4 else 4)
        for n, key in ((nthr, "dct%d_quant_blocks_per_s" % t), (1, "dct%d_quant_blocks_per_s_1t" % t)):
            res[key] = bounded(lambda n=n, t=t, mf=mf, bs=bs: orc.mb_dct_quant_mt(
                t, fenc, origin, stride, ref, origin, stride, mbw, mbh, mf, bs, n)[2], blocks)[0]
    # SATD 8x8 qpel candidates as the GPU leg scores them: per 8x8 block the +-1 qpel
    # neighbourhood of the half-pel centre (3.5, 2) px, get_ref from the ref's hpel planes
    H = mbh * 16
    hp = orc.frame_filter(8, ref, origin, stride, mbw * 16, H)
    ys, xs = np.meshgrid(np.arange(mbh * 2), np.arange(mbw * 2), indexing="ij")
    bx, by = (xs.ravel() * 8).astype(np.int64), (ys.ravel() * 8).astype(np.int64)
    fo = np.repeat(origin + by * stride + bx, 9)
    qxy = np.stack([4 * bx + 14, 4 * by + 8], 1).astype(np.int32)
    qxy = (qxy[:, None, :] + np.array([[dx, dy] for dy in (-1, 0, 1) for dx in (-1, 0, 1)], np.int32)).reshape(-1, 2)
    sp_planes = [ref] + [h.ravel() for h in hp]
    for n, key in ((nthr, "satd8x8_subpel_candidates_per_s"), (1, "satd8x8_subpel_candidates_per_s_1t")):
        res[key] = bounded(lambda n=n: orc.subpel_list_mt("satd", 3, fenc, stride, sp_planes, origin, stride, fo,
                                                          qxy, n)[1], len(fo))[0]
    res.update(cpu_lookahead(orc, planes, origin, stride, mbw, mbh, nthr, bounded))
    res.update(cpu_search(orc, mbw, mbh, nthr, bounded))
    return {"value": me_rate, "unit": "SAD16x16 candidates/s", "cores": me_used, "kind": "port",
            "cpu_model": cpu_model(), "cpus_visible": share,
            "sample": "%d full 1080p frames (%d candidates) of the same workload, %d threads, %.1f s wall; "
                      "each extra leg %.1f s" % (me_calls, me_calls * mbw * mbh * cand_per_mb, me_used, me_dt,
                                                 seconds),
            "extra": res}


if __name__ == "__main__":
    main()
