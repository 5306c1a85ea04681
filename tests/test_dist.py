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


@pytest.mark.parametrize("world,total", [(2, 4096), (2, 4097), (3, 1000)])
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


def test_shard_range_matches_appendix_b_shards(golden):
    import bench
    for k in range(8):
        g = golden["digests"][f"8Mx1500_shard{k}"]
        assert bench.shard_range(8 << 20, 8, k) == (g["seg0"], g["n"])
