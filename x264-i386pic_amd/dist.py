"""Frame-per-GPU sharding: one process per GPU, every rank owns a
contiguous slice of the (fenc, ref) frame pairs of one sequence; the search
and the residual transform of a pair need nothing from another rank, so the
data path has no collective.  The only cross-rank traffic is the benchmark's
barrier and its max-over-ranks of the timed region.

Works with any torch.distributed backend (``nccl`` = RCCL on the GPU box,
``gloo`` in the CPU tests)."""


def frame_shard(total_pairs, world, rank):
    """[start, stop) of the frame pairs owned by `rank` (contiguous, balanced:
    the first total_pairs % world ranks get one extra pair)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total_pairs, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def reduce_max(value, device="cpu"):
    """max of a python float over all ranks (identity without a process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


class LaunchError(ValueError):
    """bench.py was asked for a world it cannot run."""


def launch_plan(gpus, env, visible_devices):
    """How `bench.py --gpus N` runs (the reference's analogue is one frame thread per
    frame in flight, encoder.c:1758-1772; here one process per GPU).

    gpus            -- the --gpus argument (None: not given)
    env             -- the process environment (WORLD_SIZE set = started by a launcher)
    visible_devices -- torch.cuda.device_count() (does not initialise HIP)

    Returns ("rank", world) when this process is already one rank of a launched world,
    ("single", 1) for one process, ("spawn", n) when this process must start n rank
    processes itself.  Raises LaunchError when the request cannot be met: more RCCL ranks
    than visible GPUs (ranks may share a GPU only with X264HIP_DIST_BACKEND=gloo, which
    exercises the N > 1 path functionally and is no measurement), a --gpus that differs
    from the launcher's WORLD_SIZE, or N < 1."""
    backend = env.get("X264HIP_DIST_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise LaunchError("X264HIP_DIST_BACKEND must be nccl or gloo, not %r" % backend)
    if gpus is not None and gpus < 1:
        raise LaunchError("--gpus must be >= 1")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            raise LaunchError("--gpus %d but the launcher started WORLD_SIZE=%d ranks" % (gpus, world))
        if world > 1 and backend == "nccl" and world > visible_devices:
            raise LaunchError("%d RCCL ranks but %d visible GPUs" % (world, visible_devices))
        return ("rank", world) if world > 1 else ("single", 1)
    n = 1 if gpus is None else gpus
    if n == 1:
        return ("single", 1)
    if backend == "nccl" and n > visible_devices:
        raise LaunchError("--gpus %d but %d visible GPUs (X264HIP_DIST_BACKEND=gloo shares one GPU "
                          "between ranks for a functional run)" % (n, visible_devices))
    return ("spawn", n)


def rank_envs(n, port, base_env):
    """Environments of the n rank processes a launching bench.py starts (the variables
    torchrun would set; rendezvous on 127.0.0.1, the container hostname may not resolve)."""
    out = []
    for r in range(n):
        e = dict(base_env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out.append(e)
    return out


def spawn_ranks(argv, n, base_env, python=None, timeout=None):
    """Start n rank processes of `argv` (a script and its arguments) as children and
    wait for them.  The caller must not have touched the GPU (a child, never an exec).
    Returns the first non-zero exit code (the other ranks are then terminated) or 0."""
    import socket
    import subprocess
    import sys
    import time
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([python or sys.executable] + list(argv), env=e)
             for e in rank_envs(n, port, base_env)]
    t0 = time.monotonic()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
        if rc != 0 or (timeout is not None and time.monotonic() - t0 > timeout):
            for p in live:
                p.terminate()
            for p in live:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            if rc == 0:
                rc = 124
            break
        time.sleep(0.05)
    return rc
