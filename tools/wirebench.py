#!/usr/bin/env python3
"""Device-resident throughput of the ragged-descriptor and IPv4 wire kernels.

  * tcpcsum_batch_desc_dev on 1M segments with IMIX-like lengths
    (7:4:1 of 64 B, 576 B, 1500 B, random offsets in a 1.5 GB region);
  * tcpcsum_ipv4_batch_dev FILL and VERIFY on 1M IPv4/TCP packets of 1500 B
    in 1536-B slots (the reference's packets, device-resident).
Algorithmic bytes = the TCP segment bytes summed (+ the IP headers read for
the wire path, not counted). JSON lines.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import tcp_amd

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()

    def timeit(fn, steps=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps * 1e-3

    rng = np.random.default_rng(0)
    n = 1 << 20
    region = 1536 * n
    data = torch.empty(region, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(data, 0, region)
    lens = rng.choice(np.array([64, 576, 1500], np.uint32), n, p=[7 / 12, 4 / 12, 1 / 12])
    desc = np.zeros(n, tcp_amd.DESC_DTYPE)
    desc["offset"] = np.arange(n, dtype=np.uint64) * 1536 + rng.integers(0, 8, n).astype(np.uint64) * 4
    desc["len"] = lens
    desc["sum_start"] = rng.integers(0, 393211, n, dtype=np.uint32)
    ddesc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    for sorted_ in (False, True):
        if sorted_:   # same segments, sorted by length (how a caller can bin a batch)
            order = np.argsort(lens, kind="stable")
            d2 = desc[order]
            ddesc = torch.from_numpy(d2.view(np.uint8)).to(dev)
        for un in ((1, 2, 4) if "--sweep" in sys.argv else (0,)):
            tcp_amd.set_tuning(0, un, -1, 0)
            t = timeit(lambda: tcp_amd.batch_desc(data, ddesc, n, 1500, out))
            print(json.dumps({"measure": "desc_imix_1M", "sorted_by_len": sorted_, "unroll": un,
                              "ms": round(t * 1e3, 4), "GB/s": round(int(lens.sum()) / t / 1e9, 1),
                              "Mseg/s": round(n / t / 1e6, 1)}), flush=True)
        tcp_amd.set_tuning(0, 0, -1, 0)

    # wire: 1M packets of 1500 B (IP 20 + TCP 24 + 1456 payload) in 1536-B slots
    payload = torch.empty(n * 1456, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, n * 1456)
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = np.arange(n, dtype=np.uint64) * 1456
    segs["out_off"] = np.arange(n, dtype=np.uint64) * 1536
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"] = 4000, 45001, 1456
    segs["flags"] = 1 | 16
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, 1456, data, 0, None)
    offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * 1536).view(np.int64)).to(dev)
    stat = torch.empty(n, dtype=torch.uint8, device=dev)
    for name, mode in (("FILL", tcp_amd.IPV4_FILL), ("VERIFY", tcp_amd.IPV4_VERIFY)):
        for mb, un in (((1024, 1), (1024, 2), (2048, 2), (4096, 2), (2048, 4), (8192, 1)) if "--sweep" in sys.argv
                       else ((0, 0),)):
            tcp_amd.set_tuning(mb, un, -1, 0)
            t = timeit(lambda: tcp_amd.ipv4_batch(data, offs, n, 1536, mode, out, stat))
            print(json.dumps({"measure": "ipv4_1Mx1500", "mode": name, "max_blocks": mb, "unroll": un,
                              "ms": round(t * 1e3, 4), "GB/s_tcp_bytes": round(n * 1480 / t / 1e9, 1),
                              "Mpkt/s": round(n / t / 1e6, 1)}), flush=True)
        tcp_amd.set_tuning(0, 0, -1, 0)
    ok = bool((out == 0).all().item()) and bool((stat == 0).all().item())
    print(json.dumps({"measure": "ipv4_verify_all_zero", "ok": ok}))


if __name__ == "__main__":
    main()
