"""CPU, world_size 2 over gloo: the frame-per-GPU sharding of bench.py / x264hip.dist.

Each rank builds only its own slice of the synthetic sequence and reduces its
checksum and timing with the real torch.distributed calls the GPU run uses
(backend gloo instead of nccl); rank 0 checks that the shards partition the
sequence exactly and that the max-over-ranks reduction is right."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, load_package


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = load_package()
    from x264hip import dist as xd, synth
    start, stop = xd.frame_shard(total, world, rank)
    planes, _, _ = synth.make_sequence(stop - start + 1, 64, 32, 8, start=start)   # + the ref of the first pair
    sums = torch.tensor([int(planes[i].astype(np.int64).sum()) for i in range(len(planes))], dtype=torch.int64)
    gathered = [torch.zeros(total + 1, dtype=torch.int64) for _ in range(world)]
    padded = torch.full((total + 1,), -1, dtype=torch.int64)
    padded[start:stop + 1] = sums
    dist.all_gather(gathered, padded)
    xd.barrier()
    mx = xd.reduce_max(10.0 * (rank + 1))
    if rank == 0:
        q.put(([g.numpy() for g in gathered], mx))
    dist.destroy_process_group()
    del x


def test_frame_shard_partitions():
    x = load_package()
    from x264hip import dist as xd
    for total in (1, 7, 16, 128):
        for world in (1, 2, 3, 8):
            spans = [xd.frame_shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        xd.frame_shard(4, 2, 2)


def test_gloo_world2_shards_and_max():
    total, world = 6, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, mx = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x = load_package()
    from x264hip import synth
    full, _, _ = synth.make_sequence(total + 1, 64, 32, 8)
    want = np.array([int(f.astype(np.int64).sum()) for f in full])
    merged = np.full(total + 1, -1)
    for g in gathered:
        sel = g >= 0
        merged[sel] = g[sel]
    assert np.array_equal(merged, want)   # shards reproduce the single-process sequence
    assert mx == 20.0


def test_launch_plan_world_logic():
    """bench.py --gpus N: the parent spawns N ranks itself unless a launcher set WORLD_SIZE;
    more RCCL ranks than GPUs, or --gpus != WORLD_SIZE, is refused."""
    load_package()
    from x264hip import dist as xd
    P = xd.launch_plan
    assert P(None, {}, 0) == ("single", 1)
    assert P(1, {}, 8) == ("single", 1)
    assert P(8, {}, 8) == ("spawn", 8)
    assert P(2, {}, 2) == ("spawn", 2)
    with pytest.raises(xd.LaunchError):
        P(8, {}, 1)                                     # one GPU, eight RCCL ranks
    with pytest.raises(xd.LaunchError):
        P(0, {}, 1)
    assert P(2, {"X264HIP_DIST_BACKEND": "gloo"}, 1) == ("spawn", 2)
    assert P(8, {"X264HIP_DIST_BACKEND": "gloo"}, 0) == ("spawn", 8)
    with pytest.raises(xd.LaunchError):
        P(2, {"X264HIP_DIST_BACKEND": "mpi"}, 8)
    # started by torchrun: this process is one rank
    assert P(4, {"WORLD_SIZE": "4"}, 8) == ("rank", 4)
    assert P(None, {"WORLD_SIZE": "4"}, 8) == ("rank", 4)
    assert P(None, {"WORLD_SIZE": "1"}, 1) == ("single", 1)
    with pytest.raises(xd.LaunchError):
        P(8, {"WORLD_SIZE": "4"}, 8)
    with pytest.raises(xd.LaunchError):
        P(4, {"WORLD_SIZE": "4"}, 2)
    assert P(4, {"WORLD_SIZE": "4", "X264HIP_DIST_BACKEND": "gloo"}, 1) == ("rank", 4)
    envs = xd.rank_envs(3, 1234, {"A": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "1234"
               and e["A"] == "1" for e in envs)


_RANK_SCRIPT = r'''
import json, os, sys
import torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
got = [None] * w
dist.all_gather_object(got, int(os.environ["LOCAL_RANK"]))
if r == 0:
    print(json.dumps({"world": w, "locals": got}))
if r == 1 and len(sys.argv) > 1 and sys.argv[1] == "fail":
    sys.exit(3)
dist.destroy_process_group()
'''


def test_spawn_ranks_gloo(tmp_path, capfd):
    """spawn_ranks starts real ranks that rendezvous over gloo on 127.0.0.1, and a failing
    rank's exit code comes back to the parent."""
    load_package()
    from x264hip import dist as xd
    import json
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    assert xd.spawn_ranks([str(script)], 3, env, timeout=120) == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert json.loads(out[-1]) == {"world": 3, "locals": [0, 1, 2]}
    assert xd.spawn_ranks([str(script), "fail"], 2, env, timeout=120) == 3


def test_bench_refuses_more_ranks_than_gpus():
    """`python bench.py --gpus 8` on a host with fewer GPUs exits non-zero before any GPU work."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "X264HIP_DIST_BACKEND")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2
    assert "visible GPUs" in p.stderr
