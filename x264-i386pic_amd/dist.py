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
