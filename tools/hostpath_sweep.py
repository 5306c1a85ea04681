#!/usr/bin/env python3
"""Staged host paths (pageable memory copied into pinned staging) under the
context's copy knobs, read at tcpcsum_ctx_create:
  TCPCSUM_HOST_THREADS       copy threads (incl. the caller's)
  TCPCSUM_HOST_NT            streaming stores for the uniform chunks
  TCPCSUM_HOST_DMA           uniform chunks: DMA to HBM then the kernel (0: kernel reads staging over PCIe)
  TCPCSUM_HOST_SPIN_US       how long an idle copy thread spins before it sleeps
  TCPCSUM_HOST_STAGE_PASSES  wire staging: 1 = laid out by bounds, one pass; 2 = lengths first, packed
  TCPCSUM_HOST_NUMA          copy threads on the GPU's NUMA node (0: anywhere)
--configs: threads:nt:dma[:spin_us[:passes[:numa]]],...
Wire packets are staged on the copy threads (header reads, copies and the FILL
write-back) and checksummed by one launch.
Measures tcpcsum_batch_uniform_host over 1M x 1500 B pageable, and one
releaseSend batch (1024 x 1500-B packets) FILLed through
tcpcsum_ipv4_batch_host (pageable 32 KiB-slot pool) and
tcpcsum_ipv4_batch_ptrs_host (1024 separate pageable 32 KiB buffers, the
loop's layout, loop.c:180-183), with the context's copy / wait split.
Interleaved rounds; one JSON line per (config, measure, round).

  python tools/hostpath_sweep.py [--rounds 2]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--configs", default="8:1:1:50:1:0,8:1:1:50:1:1,4:1:1:50:1:0,4:1:1:50:1:1")
    ap.add_argument("--wire-only", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import tcp_amd
    from tests.packets import ip_packet
    rng = np.random.default_rng(3)
    n, L = 1 << 20, 1500
    big = np.empty(n * L, np.uint8)
    big[:] = rng.integers(0, 256, big.size, dtype=np.uint8)
    ss = rng.integers(0, 393211, n, dtype=np.uint32)
    want = None
    pkts = [np.frombuffer(ip_packet(rng, 1456), np.uint8) for _ in range(1024)]
    pool = np.zeros(1024 * 32768, np.uint8)
    for i, p in enumerate(pkts):
        pool[i * 32768:i * 32768 + p.size] = p
    offs = np.arange(1024, dtype=np.uint64) * 32768
    bufs = []
    for i in range(2048):   # separate allocations, every other one a packet buffer
        b = np.empty(32768, np.uint8)
        if i & 1:
            b[:1500] = pkts[i // 2]
        bufs.append(b)
    ptrs = np.array([b.ctypes.data for b in bufs[1::2]], np.uint64)   # arrays, not lists: no per-call conversion
    lens = np.full(1024, 1500, np.uint32)
    defaults = [8, 1, 1, 50, 1, 1]
    configs = []
    for c in args.configs.split(","):
        v = [int(x) for x in c.split(":")]
        configs.append(tuple(v + defaults[len(v):]))
    # one core's memcpy of the batch's 1.5 MB into pageable vs page-locked memory (is the
    # staging itself slow to write?)
    import ctypes
    src = np.frombuffer(rng.bytes(1536000), np.uint8).copy()
    dst_pg = np.empty(1536000, np.uint8)
    dst_pin = tcp_amd.pinned_empty(1536000)
    for name, dst in (("pageable", dst_pg), ("pinned", dst_pin)):
        dst[:] = 0
        tmin, tmed = timed(lambda: ctypes.memmove(dst.ctypes.data, src.ctypes.data, src.size), 200)
        print(json.dumps({"measure": "memcpy_1p5MB_one_core", "dst": name, "us_median": round(tmed * 1e6, 1),
                          "us_best": round(tmin * 1e6, 1), "GB/s_median": round(src.size / tmed / 1e9, 2)}),
              flush=True)
    for rnd in range(args.rounds):
        for th, nt, dma, spin, passes, numa in configs:
            os.environ["TCPCSUM_HOST_THREADS"] = str(th)
            os.environ["TCPCSUM_HOST_NT"] = str(nt)
            os.environ["TCPCSUM_HOST_DMA"] = str(dma)
            os.environ["TCPCSUM_HOST_SPIN_US"] = str(spin)
            os.environ["TCPCSUM_HOST_STAGE_PASSES"] = str(passes)
            os.environ["TCPCSUM_HOST_NUMA"] = str(numa)
            with tcp_amd.HostContext(0) as ctx:
                cfg = {"threads": th, "nt": nt, "dma": dma, "spin_us": spin, "passes": passes, "numa": numa,
                       "round": rnd}
                if args.wire_only:
                    pass
                else:
                    got = ctx.batch_uniform(big, L, L, n, ss)
                    if want is None:
                        want = got
                    assert np.array_equal(got, want)
                    s0 = ctx.stats()
                    tmin, tmed = timed(lambda: ctx.batch_uniform(big, L, L, n, ss), 5)
                    s1 = ctx.stats()
                    print(json.dumps({**cfg, "measure": "uniform_host_1Mx1500_pageable",
                                      "GiB/s_median": round(n * L / tmed / 2**30, 2),
                                      "GiB/s_best": round(n * L / tmin / 2**30, 2),
                                      "copy_ms_per_call": round((s1["ns_copy"] - s0["ns_copy"]) / 5e6, 3),
                                      "wait_ms_per_call": round((s1["ns_wait"] - s0["ns_wait"]) / 5e6, 3)}),
                          flush=True)
                for name, fn in (("ipv4_host_pool32k_fill", lambda: ctx.ipv4_batch(pool, offs, 32768, 0)),
                                 ("ipv4_ptrs_host_loop_fill", lambda: ctx.ipv4_batch_ptrs(ptrs, lens, 0))):
                    fn()
                    s0 = ctx.stats()
                    reps = 300
                    tmin, tmed = timed(fn, reps)
                    s1 = ctx.stats()
                    print(json.dumps({**cfg, "measure": name, "us_median": round(tmed * 1e6, 1),
                                      "us_best": round(tmin * 1e6, 1),
                                      "copy_us_per_call": round((s1["ns_copy"] - s0["ns_copy"]) / reps / 1e3, 1),
                                      "wait_us_per_call": round((s1["ns_wait"] - s0["ns_wait"]) / reps / 1e3, 1)}),
                          flush=True)


if __name__ == "__main__":
    main()
