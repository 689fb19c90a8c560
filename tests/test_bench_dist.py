"""bench.py's multi-GPU logic on CPU: world_size-2 gloo ranks (replicas, weak
scaling, one MAX reduction of the timed-region seconds, no data-path
collective)."""
import os
import socket
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank: int, world: int, port: int, q) -> None:
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        elapsed = 1.0 + 0.5 * rank  # rank 1 is the slow one
        job = bench.max_over_ranks(elapsed, dist, "cpu")
        ids = bench.clip_ids(rank, 4, 1, 2)
        q.put((rank, job, ids))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_max_reduce():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    assert [o[1] for o in out] == [1.5, 1.5]  # every rank sees the max
    flat = [c for o in out for step in o[2] for c in step]
    assert len(flat) == len(set(flat)) == 2 * 3 * 4  # disjoint clips, 3 steps x 4 clips per rank


def test_job_value_is_whole_job_aggregate():
    import bench

    assert bench.job_rtf(8, 32, 2, 2.0) == pytest.approx(8 * 32 * 2 * 30.0 / 2.0)
    assert bench.max_over_ranks(3.25, None, "cpu") == 3.25
    assert bench.clip_ids(0, 2, 1, 1) == [[0, 1], [2, 3]]
    assert bench.clip_ids(1, 2, 1, 1) == [[4, 5], [6, 7]]


def _init_rank(rank: int, world: int, port: int, q) -> None:
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import bench

    dist = bench.init_dist()
    try:
        job = bench.max_over_ranks(2.0 + rank, dist, "cpu")
        q.put((rank, dist.get_backend(), job))
    finally:
        dist.destroy_process_group()


def test_bench_group_is_gloo_not_rccl():
    """The bench's own group constructor: a host (gloo) group, never NCCL/RCCL
    (north_star 'RCCL unused')."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_init_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[1] for o in out] == ["gloo", "gloo"]
    assert [o[2] for o in out] == [3.0, 3.0]
    src = open(os.path.join(REPO, "bench.py")).read()
    assert '"nccl"' not in src and "'nccl'" not in src
