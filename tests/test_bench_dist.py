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


def _bench_env() -> dict:
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` with no torch.distributed.run environment
    starts 2 rank processes itself (gloo group), and rank 0's one JSON line
    says n_gpus = 2."""
    import json
    import subprocess

    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "2",
                          "--warmup", "1", "--clips-per-gpu", "4"], env=_bench_env(), capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(s) for s in out.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2 and line["backend"] == "gloo"
    assert line["clips_rank0"] == 3 * 4
    assert line["value"] == pytest.approx(2 * 4 * 2 * 30.0 / (line["ms_per_step"] * 2e-3), rel=1e-2)


def test_bench_gpus_rank_failure_stops_the_others():
    """One rank of `bench.py --gpus 2` exits with status 3 before the
    rendezvous (test-only BENCH_DRY_RUN_FAIL): the other rank would wait in
    init_process_group forever, so launch_ranks must terminate it and return
    the failing rank's status."""
    import re
    import subprocess
    import time

    env = dict(_bench_env(), BENCH_DRY_RUN_FAIL="1:3")
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert "rank 1 exited with status 3" in out.stderr
    assert time.time() - t0 < 200  # rank 0 was stopped, not left waiting for the rendezvous timeout
    pids = {int(r): int(p) for r, p in re.findall(r"rank (\d) pid (\d+)", out.stderr)}
    assert sorted(pids) == [0, 1]
    for pid in pids.values():  # both children are gone (reaped by launch_ranks)
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)
    assert not any(s.startswith("{") for s in out.stdout.splitlines())  # no JSON line from a failed job


def test_bench_one_gpu_dry_run_and_mismatch():
    import json
    import subprocess

    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run"], env=_bench_env(),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["n_gpus"] == 1
    # a torch.distributed.run environment that disagrees with --gpus is refused before any GPU call
    env = dict(_bench_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    bad = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                         capture_output=True, text=True, timeout=240)
    assert bad.returncode == 2 and "WORLD_SIZE=1" in bad.stderr
