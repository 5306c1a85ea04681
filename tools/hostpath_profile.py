#!/usr/bin/env python3
"""One releaseSend batch (1024 x 1500-B packets) through the two zero-copy host
paths, for a rocprofv3 kernel trace that tells kernel time from host time:

  * tcpcsum_ipv4_batch_host on a pinned pool (32 KiB slots, tcpcsum_host_alloc)
  * tcpcsum_ipv4_batch_ptrs_host on 1024 separate pageable 32 KiB buffers
    (page-locked on first use; loop.c:180-183)

Both launch k_ipv4<16,2,1,...>; the scatter-gather one is the PL=true
instantiation, so the trace separates them. Prints per-path wall medians.

  rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/hostpath_profile.py
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import tcp_amd
    from tests.packets import ip_packet

    rng = np.random.default_rng(2)
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    ctx = tcp_amd.HostContext(0)
    pool = tcp_amd.pinned_empty(1024 * 32768)
    offs = np.arange(1024, dtype=np.uint64) * np.uint64(32768)
    bufs = []
    for i in range(2048):
        b = np.empty(32768, np.uint8)
        if i & 1:
            p = np.frombuffer(ip_packet(rng, 1456), np.uint8)
            b[:p.size] = p
            k = i // 2
            pool[k * 32768:k * 32768 + p.size] = p
        bufs.append(b)
    ptrs = np.array([b.ctypes.data for b in bufs[1::2]], np.uint64)
    lens = np.full(1024, 1500, np.uint32)
    res = {}
    for name, fn in (("pinned_pool_region", lambda: ctx.ipv4_batch(pool, offs, 32768, tcp_amd.IPV4_FILL)),
                     ("ptrs_pageable_buffers", lambda: ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL))):
        fn()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[name] = {"us_median": round(statistics.median(ts) * 1e6, 1), "us_min": round(min(ts) * 1e6, 1)}
    # latency floor: the same call on 1 and 64 packets (launch + synchronize + host work)
    for k in (1, 64, 256):
        fn = lambda: ctx.ipv4_batch_ptrs(ptrs[:k], lens[:k], tcp_amd.IPV4_FILL)
        fn()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[f"ptrs_{k}_packets"] = {"us_median": round(statistics.median(ts) * 1e6, 1),
                                    "us_min": round(min(ts) * 1e6, 1)}
    ctx.close()
    print(json.dumps({"measure": "host_zero_copy_paths_1024x1500", "iters": iters, **res}))


if __name__ == "__main__":
    main()
