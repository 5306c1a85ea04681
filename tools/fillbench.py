#!/usr/bin/env python3
"""Wire kernel variants on MI355X: tuning flags 0 (128-B windows, nt loads),
32 (WIRE_CACHED: default-policy loads), 64 (WIN16: 16-B windows), 96 (both).

1M IPv4/TCP packets of 1500 B in 1536-B slots, device-resident, the slots
64-B aligned (base) and 16-B aligned (base + 16, the reference's malloc'd
buffers are only 16-B aligned). Reports kernel time (HIP events) per flag.
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
    n, slot = 1 << 20, 1536
    payload = torch.empty(n * 1456, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, n * 1456)
    data = torch.empty(n * slot + 64, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    stat = torch.empty(n, dtype=torch.uint8, device=dev)
    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 20)
        return sorted(ts)[1]

    for shift in (0, 16, 80):
        segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
        segs["payload_off"] = np.arange(n, dtype=np.uint64) * 1456
        segs["out_off"] = np.arange(n, dtype=np.uint64) * slot + shift
        segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
        segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, 1456, 1 | 16
        tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, 1456, data, 0, None)
        offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * slot + shift).view(np.int64)).to(dev)
        for flags in (0, 32, 64, 96):
            tcp_amd.set_tuning(0, 0, -1, flags)
            fn = lambda: tcp_amd.ipv4_batch(data, offs, n, slot, tcp_amd.IPV4_VERIFY, out, stat)
            ms = timed(fn)
            print(json.dumps({"measure": "ipv4_verify_1Mx1500", "slot_shift": shift, "flags": flags,
                              "ms": round(ms, 4), "GB/s_tcp_bytes": round(n * 1480 / (ms * 1e-3) / 1e9, 1)}),
                  flush=True)
            tcp_amd.set_tuning(0, 0, -1, 0)
        for iphdr in (0, tcp_amd.IPV4_IPHDR):
            for flags in (0, 32, 64, 96):
                tcp_amd.set_tuning(0, 0, -1, flags)
                fn = lambda: tcp_amd.ipv4_batch(data, offs, n, slot, tcp_amd.IPV4_FILL | iphdr, out, stat)
                ms = timed(fn)
                tcp_amd.set_tuning(0, 0, -1, 0)
                tcp_amd.ipv4_batch(data, offs, n, slot, tcp_amd.IPV4_VERIFY | iphdr, out, stat)
                ok = bool((out == 0).all().item()) and bool((stat == 0).all().item())
                print(json.dumps({"measure": "ipv4_fill_1Mx1500", "slot_shift": shift, "iphdr": bool(iphdr),
                                  "flags": flags, "ms": round(ms, 4),
                                  "GB/s_tcp_bytes": round(n * 1480 / (ms * 1e-3) / 1e9, 1), "verify_ok": ok}),
                      flush=True)


if __name__ == "__main__":
    main()
