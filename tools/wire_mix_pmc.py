#!/usr/bin/env python3
"""Dispatch sequence for PMC passes over the balanced wire kernel on bench.py's flush mix:
10 VERIFYs, 10 FILLs (k_ipv4_lb, told apart by dispatch order), 10 read-only probes over the same
region (k_probe), then 10 VERIFYs of 1M x 1500-B packets in 1536-B slots (the lane-group kernel
k_ipv4) for comparison. Prints the bytes each dispatch group reads (TCP bytes / region bytes).

  rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU ... --output-format csv -d DIR -o p -- python3 tools/wire_mix_pmc.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import tcp_amd
    import bench
    dev = torch.device("cuda:0")
    n = 1 << 20
    segs, region = bench.wire_mix_segments(n)
    reg, doff, built, tcp_bytes = bench.build_wire(segs, region, 1456, dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    for mode in (tcp_amd.IPV4_VERIFY, tcp_amd.IPV4_FILL):
        for _ in range(10):
            tcp_amd.ipv4_batch(reg, doff, n, 1500, mode, out, st)
    torch.cuda.synchronize()
    assert bool(torch.equal(out, built))
    pout = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=dev)
    for _ in range(10):
        tcp_amd.stream_probe(reg, (region // 16) * 16, pout, tune=(0, 0, -1, 0))
    torch.cuda.synchronize()
    del reg
    segs2 = segs.copy()
    import numpy as np
    segs2["out_off"] = np.arange(n, dtype=np.uint64) * 1536
    segs2["len"], segs2["flags"] = 1456, 17
    reg2, doff2, _, tcp2 = bench.build_wire(segs2, n * 1536, 1456, dev)
    for _ in range(10):
        tcp_amd.ipv4_batch(reg2, doff2, n, 1536, tcp_amd.IPV4_VERIFY, out, st)
    torch.cuda.synchronize()
    print(json.dumps({"mix_tcp_bytes": tcp_bytes, "mix_region_bytes": region, "mtu_tcp_bytes": tcp2,
                      "groups": ["mix VERIFY x10", "mix FILL x10", "probe x10", "MTU VERIFY x10"]}))


if __name__ == "__main__":
    main()
