#!/usr/bin/env python3
"""Byte-granular paths (odd starts / odd lengths), device-resident: kernel time
per workload for the library at $TCPCSUM_LIB (A/B of two builds: run once per
build). The two builds' outputs are compared by the caller: every workload
prints an fnv1a64 of its first 64 KiB of results. Workloads:

  * uniform M1: 1M segments of 1499 B at stride 1499 (odd starts and lengths);
  * uniform long M1: 64K segments of 16383 B at stride 16385;
  * ragged lane groups (forced shape 4, 64 chunks): 256K segments of 1499 B at
    odd offsets, random order.
(The wire kernel at odd packet addresses is A/B'd by tools/wire_ab.py and
tools/wiresweep.py, not here.)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def fnv(a):
    import numpy as np
    h = 0xcbf29ce484222325
    for b in a.astype("<u2").tobytes()[:1 << 16]:
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return hex(h)


def main():
    import numpy as np
    import torch
    import tcp_amd

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    tag = os.environ.get("AB_TAG", "cur")

    def timeit(fn, steps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(steps):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / steps)
        return sorted(ts)[2]

    nbytes = (1 << 20) * 1537 + 4096
    data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(data, 0, nbytes)

    def report(name, ms, alg, outt):
        h = fnv(outt.cpu().numpy().view(np.uint16))
        print(json.dumps({"lib": tag, "measure": name, "ms": round(ms, 4),
                          "GB/s": round(alg / (ms * 1e-3) / 1e9, 1), "fnv_head": h}), flush=True)

    n, L = 1 << 20, 1499
    out = torch.empty(n, dtype=torch.int16, device=dev)
    ms = timeit(lambda: tcp_amd.batch_uniform(data, L, L, n, 12345, out=out, offset=1))
    report("uniform_M1_1Mx1499", ms, n * L, out)

    n2, L2, S2 = 1 << 16, 16383, 16385
    out2 = torch.empty(n2, dtype=torch.int16, device=dev)
    ms = timeit(lambda: tcp_amd.batch_uniform(data, S2, L2, n2, 777, out=out2, offset=3))
    report("uniform_M1_64Kx16383", ms, n2 * L2, out2)

    n3 = 1 << 18
    rng = np.random.default_rng(7)
    offs = rng.permutation(n3).astype(np.uint64) * 1504 + 1
    desc = np.zeros(n3, tcp_amd.DESC_DTYPE)
    desc["offset"], desc["len"], desc["sum_start"] = offs, 1499, rng.integers(0, 1 << 20, n3)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    out3 = torch.empty(n3, dtype=torch.int16, device=dev)
    for sh in (-1, 4):
        tcp_amd.set_tuning(0, 0, sh, 0)
        ms = timeit(lambda: tcp_amd.batch_desc(data, d_desc, n3, 1499, out=out3))
        report(f"desc_shape{sh}_256Kx1499_odd", ms, n3 * 1499, out3)
    tcp_amd.set_tuning(0, 0, -1, 0)


if __name__ == "__main__":
    main()
