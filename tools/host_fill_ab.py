#!/usr/bin/env python3
"""In-place host FILL: the check's store shape and the kernel shape for one releaseSend batch
(1024 x 1500-B packets, one per 32 KiB slot of a page-locked pool, loop.c:180-183 layout) through
tcpcsum_ipv4_batch_ptrs_host — the interposer's call. Variants interleaved in rounds, wall time
per call (sleeping wait, as the interposer waits). Every variant's packets must equal the oracle's
FILL. JSON lines.

  python tools/host_fill_ab.py
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch  # noqa: F401  (the HIP runtime the library binds to)
    import tcp_amd
    import oracle
    from tests.packets import ip_packet
    n, slot = 1024, 32768
    rng = np.random.default_rng(5)
    pool = tcp_amd.pinned_empty(n * slot)
    pool[:] = 0
    pkts = [ip_packet(rng, 1456) for _ in range(n)]
    for i, p in enumerate(pkts):
        pool[i * slot:i * slot + len(p)] = np.frombuffer(p, np.uint8)
    want = pool.copy()
    offs = np.arange(n, dtype=np.uint64) * slot
    oracle.ipv4_batch(want, offs, 65535, tcp_amd.IPV4_FILL)
    ptrs = [pool.ctypes.data + i * slot for i in range(n)]
    lens = np.array([len(p) for p in pkts], np.uint32)
    variants = {}
    for shape in (-1, 0, 4, 6, 7):
        for name, fl in (("line", 0), ("u16", tcp_amd.TUNE_FILL_U16)):
            variants[f"shape{shape}_{name}"] = (shape, fl)
    ctx = tcp_amd.HostContext(0, blocking_wait=True)
    times = {k: [] for k in variants}
    same = {}
    for k, (shape, fl) in variants.items():
        ctx.set_tuning(0, 0, shape, fl)
        for i in range(n):   # check = 0 again, then FILL
            pool[i * slot + 36:i * slot + 38] = 0
        ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL)
        same[k] = bool(np.array_equal(pool, want))
    for _ in range(int(os.environ.get("ROUNDS", "4"))):
        for k, (shape, fl) in variants.items():
            ctx.set_tuning(0, 0, shape, fl)
            for _ in range(5):
                ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL)
            for _ in range(60):
                t0 = time.perf_counter()
                ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL)
                times[k].append((time.perf_counter() - t0) * 1e6)
    st = ctx.stats()
    ctx.close()
    for k, ts in times.items():
        print(json.dumps({"variant": k, "us_median": round(statistics.median(ts), 1), "us_min": round(min(ts), 1),
                          "same_as_oracle": same[k]}), flush=True)
    print(json.dumps({"pkts_in_place": st["pkts_in_place"], "pkts_staged": st["pkts_staged"]}))


if __name__ == "__main__":
    main()
