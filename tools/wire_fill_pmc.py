#!/usr/bin/env python3
"""Dispatch sequence for a WRITE_SIZE / FETCH_SIZE pass over the wire FILL stores:
1M x 1500-B packets in 1536-B slots (device), 10 FILLs with the 2-byte store
(TCPCSUM_TUNE_FILL_U16), then 10 FILLs with the default line store, then 10
VERIFYs — in that order, so the rows of a rocprofv3 --pmc run (same kernel
name for all three) are told apart by dispatch order — then 10 launches of the
write-back probe over the same region (k_probe<8, true>: exactly 1M x 1536 B
read and 1M x 128 B written through), the counters' calibration.

  rocprofv3 --pmc WRITE_SIZE --output-format csv -d DIR -o p -- python3 tools/wire_fill_pmc.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import tcp_amd
    dev = torch.device("cuda:0")
    n, slot = 1 << 20, 1536
    payload = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, payload.numel())
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = (np.arange(n, dtype=np.uint64) * 4096) % np.uint64(payload.numel() - 65536)
    segs["out_off"] = np.arange(n, dtype=np.uint64) * slot
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, 1456, 1 | 16
    reg = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, 1456, reg, 0, None)
    off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    out = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    u16 = tcp_amd.make_tuning(0, 0, -1, tcp_amd.TUNE_FILL_U16)
    for _ in range(10):
        tcp_amd.ipv4_batch(reg, off, n, slot, 0, out, st, tune=u16)
    for _ in range(10):
        tcp_amd.ipv4_batch(reg, off, n, slot, 0, out, st)
    for _ in range(10):
        tcp_amd.ipv4_batch(reg, off, n, slot, 1, out, st)
    torch.cuda.synchronize()
    assert bool((out == 0).all().item())
    # calibration: the write-back probe moves exactly 1M x 1536 B read + 1M x 128 B written
    pout = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=dev)
    for _ in range(10):
        tcp_amd.stream_probe(reg, n * slot, pout, tune=(8192, 1, slot // 128, tcp_amd.TUNE_PROBE_WRITE))
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
