"""CPU, world_size 2 over gloo: bench.py's multi-GPU plumbing.

bench.py --gpus N runs one process per GPU; each owns a contiguous shard of
segments (bench.shard_range) and there is no collective on the data path — only
barriers around the timed region and a max-over-ranks of its duration
(bench.timed_region, bench.max_over_ranks). Here the same functions run on CPU
ranks with the oracle standing in for the per-rank kernel, and the gathered
shards must equal the unsharded batch.
"""
import os
import socket

import numpy as np
import pytest


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, seg_len, q):
    import torch
    import torch.distributed as dist

    import bench
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s0, cnt = bench.shard_range(total, world, rank)
        res = {}

        def step():
            res["out"] = oracle.synth_batch(s0, cnt, seg_len, threads=1)

        wall = bench.timed_region(step, 3, 1, dist, lambda: None)
        wmax = bench.max_over_ranks(wall, dist, torch.device("cpu"))
        outs = [None] * world
        dist.all_gather_object(outs, (s0, cnt, res["out"].tobytes(), wall, wmax))
        if rank == 0:
            q.put(outs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 4096), (2, 4097), (3, 1000), (8, 8192)])
def test_sharded_equals_unsharded_gloo(world, total):
    import torch.multiprocessing as mp

    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, 1500, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # contiguous, disjoint, covering
    starts = [o[0] for o in outs]
    cnts = [o[1] for o in outs]
    assert starts[0] == 0 and sum(cnts) == total
    assert all(starts[i] + cnts[i] == starts[i + 1] for i in range(world - 1))
    gathered = np.concatenate([np.frombuffer(o[2], np.uint16) for o in outs])
    assert np.array_equal(gathered, oracle.synth_batch(0, total, 1500))
    # every rank agrees on the max-over-ranks duration, and it is the max
    walls = [o[3] for o in outs]
    assert all(abs(o[4] - max(walls)) < 1e-12 for o in outs)


def _host_worker(rank, world, port, q):
    import torch.distributed as dist

    import bench
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the host leg's sharding (bench.run_host_path): rank r's shard of world x 4096 segments,
        # summed here by the oracle in place of the context
        total = 4096 * world
        s0, cnt = bench.shard_range(total, world, rank)
        import time
        out = {}

        def step():
            out["r"] = oracle.synth_batch(s0, cnt, 1500, threads=1)
            time.sleep(0.002)

        wall = bench.timed_region(step, 3, 1, dist, lambda: None)
        walls = bench.gather_walls(wall, dist, world)
        rate = bench.host_path_rate([cnt * 1500] * world, walls, 3)
        objs = [None] * world
        dist.all_gather_object(objs, (s0, cnt, out["r"].tobytes(), wall, walls, rate))
        if rank == 0:
            q.put(objs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_path_sharding_and_aggregation_gloo(world):
    """bench.run_host_path at N > 1 on CPU ranks: contiguous shards covering the global batch, every
    rank sees every rank's wall time, and the whole-job rate is all ranks' bytes over the slowest."""
    import torch.multiprocessing as mp

    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    objs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = 4096 * world
    gathered = np.concatenate([np.frombuffer(o[2], np.uint16) for o in objs])
    assert np.array_equal(gathered, oracle.synth_batch(0, total, 1500))
    walls = [o[3] for o in objs]
    for o in objs:
        assert o[4] == walls                                  # the same list on every rank
        assert o[5]["wall_max_s"] == round(max(walls), 6)
        assert abs(o[5]["GiB/s"] - total * 1500 * 3 / max(walls) / 2**30) < 0.01


def test_host_path_rate_single():
    import bench
    r = bench.host_path_rate([1 << 30], [0.5], 2)
    assert r["GiB/s"] == 4.0 and r["per_rank_GiB/s"] == [4.0]


def test_shard_range_matches_appendix_b_shards(golden):
    import bench
    for k in range(8):
        g = golden["digests"][f"8Mx1500_shard{k}"]
        assert bench.shard_range(8 << 20, 8, k) == (g["seg0"], g["n"])


STUB = """
import json, os, sys, time
sys.path.insert(0, {repo!r})
import torch, torch.distributed as dist
import bench
rank, world, _ = bench.dist_env()
dist.init_process_group("gloo")
if os.environ.get("STUB_FAIL_RANK") == str(rank):
    print(f"stub rank {{rank}}: simulated failure", file=sys.stderr)
    sys.exit(7)
wall = bench.timed_region(lambda: time.sleep(0.001 * (rank + 1)), 3, 1, dist, lambda: None)
wmax = bench.max_over_ranks(wall, dist, torch.device("cpu"))
if rank == 0:
    print(json.dumps({{"world": world, "wall_max": wmax, "mine": wall}}))
dist.destroy_process_group()
"""


@pytest.mark.parametrize("world", [2, 3])
def test_spawn_ranks_relays_rank0_line(tmp_path, world):
    """bench.py --gpus N without a launcher: N rank processes on 127.0.0.1, rank 0's line relayed,
    the max over ranks is the slowest rank's time."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stub = tmp_path / "stub.py"
    stub.write_text(STUB.format(repo=repo))
    code = ("import sys, argparse; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(argparse.Namespace(gpus=%d), [], script=%r))" % (repo, world, str(stub)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr
    import json
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["world"] == world and d["wall_max"] >= d["mine"] > 0


def test_spawn_ranks_stops_the_others_when_one_fails(tmp_path):
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stub = tmp_path / "stub.py"
    stub.write_text(STUB.format(repo=repo))
    code = ("import sys, argparse; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(argparse.Namespace(gpus=2), [], script=%r))" % (repo, str(stub)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["STUB_FAIL_RANK"] = "1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 7
    # the failing rank's exit code and the tail of its stderr reach the launcher's stderr
    assert "rank 1 exited with code 7 (first to fail)" in r.stderr
    assert "stub rank 1: simulated failure" in r.stderr
