#!/usr/bin/env python3
"""bench.py's wire leg (run_wire) in a process of its own, then VERIFY timed on the region the
builder wrote vs a clone of it and vs a region written by a plain copy, interleaved (diagnostic)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import bench
    import tcp_amd
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    print(json.dumps({"run_wire": bench.run_wire(20, 5, dev)}), flush=True)
    n, slot = 1 << 20, 1536
    payload = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, payload.numel())
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = (np.arange(n, dtype=np.uint64) * 4096) % np.uint64(payload.numel() - 65536)
    segs["out_off"] = np.arange(n, dtype=np.uint64) * slot
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, 1456, 1 | 16
    built = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, 1480, built, 0, None)
    regs = {"built": built, "clone": built.clone()}
    cp = torch.empty_like(built)
    cp.copy_(built)
    regs["copy_into_empty"] = cp
    doff = torch.from_numpy((np.arange(n, dtype=np.uint64) * slot).view(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    sta = torch.empty(n, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    res = {(k, m): [] for k in regs for m in (1, 0)}
    for _ in range(5):
        for k, r in regs.items():
            for m in (1, 0):
                for _ in range(3):
                    tcp_amd.ipv4_batch(r, doff, n, slot, m, out, sta)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(20):
                    tcp_amd.ipv4_batch(r, doff, n, slot, m, out, sta)
                e1.record(st)
                torch.cuda.synchronize()
                res[(k, m)].append(e0.elapsed_time(e1) / 20)
    for (k, m), t in res.items():
        print(json.dumps({"region": k, "mode": "verify" if m else "fill", "ms_median": round(statistics.median(t), 4),
                          "ms_min": round(min(t), 4)}), flush=True)


if __name__ == "__main__":
    main()
