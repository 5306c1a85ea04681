#!/usr/bin/env python3
"""Launch-shape sweep of the ragged-descriptor kernels (k_desc lane groups, k_desc_lb
balanced) on equal-length descriptor batches of several sizes, device-resident.

Each size: n descriptors of L bytes at stride L rounded up to 16 (>= 65536 of them,
>= ~1.5 GB), every start value from synth_pseudo. Interleaved rounds (every shape
once per round, median over rounds); every shape's results must equal the auto
choice's. JSON lines.

  python tools/desc_sweep.py            (SIZES / SHAPES env: comma lists; N: descriptors per batch)
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import tcp_amd
    from tests.tensors import to_dev
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    sizes = [int(x) for x in os.environ.get("SIZES", "64,1500,4096,9000,32768,65536").split(",")]
    shapes = [int(x) for x in os.environ.get("SHAPES", "-1,3,4,5,6,7,8").split(",")]
    # UNROLLS: comma list crossed with SHAPES (balanced shapes 7 / 8: at most 64 / unroll segments
    # per wave tile; 0 = the plan's)
    unrolls = [int(x) for x in os.environ.get("UNROLLS", "0").split(",")]
    variants = [(sh, u) for sh in shapes for u in unrolls]
    rounds = int(os.environ.get("ROUNDS", "5"))
    for L in sizes:
        if L == 0:   # size 0: a packed ragged batch of IMIX-like lengths 40..1500, ~1.5 GB
            lens = np.random.default_rng(5).integers(40, 1501, 1 << 22).astype(np.uint32)
            n = int(np.searchsorted(np.cumsum(lens.astype(np.uint64)), 1572864000))
            lens = lens[:n]
            offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
            data = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device=dev)
            tcp_amd.synth_fill(data, 0, data.numel())
            L = 1500   # max_len
        else:
            stride = (L + 15) & ~15
            n = int(os.environ["N"]) if os.environ.get("N") else max(65536, (3 << 29) // stride)
            data = torch.empty(n * stride, dtype=torch.uint8, device=dev)
            tcp_amd.synth_fill(data, 0, n * stride)
            offs = np.arange(n, dtype=np.uint64) * stride
            lens = np.full(n, L, np.uint32)
        d = np.zeros(n, tcp_amd.DESC_DTYPE)
        d["offset"] = offs
        d["len"] = lens
        d["sum_start"] = np.arange(n, dtype=np.uint32) * 7
        dd = to_dev(d.view(np.uint8), dev)
        outs = {v: torch.empty(n, dtype=torch.int16, device=dev) for v in variants}
        times = {v: [] for v in variants}
        for _ in range(rounds):
            for v in variants:
                sh = v
                t = tcp_amd.make_tuning(0, v[1], v[0], 0)
                for _ in range(2):
                    tcp_amd.batch_desc(data, dd, n, L, out=outs[sh], tune=t)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10):
                    tcp_amd.batch_desc(data, dd, n, L, out=outs[sh], tune=t)
                e1.record(st)
                torch.cuda.synchronize()
                times[sh].append(e0.elapsed_time(e1) / 10)
        ref = outs[variants[0]]
        for v in variants:
            ms = statistics.median(times[v])
            print(json.dumps({"measure": "desc_shape_sweep", "len": L, "n": n, "shape": v[0], "unroll": v[1],
                              "ms": round(ms, 4), "GB/s": round(int(lens.sum()) / (ms * 1e-3) / 1e9, 1),
                              "equal_to_first": bool(torch.equal(outs[v], ref))}), flush=True)
        del data, dd, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
