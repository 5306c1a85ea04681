#!/usr/bin/env python3
"""Shapes of the write-back stream probe (TCPCSUM_TUNE_PROBE_WRITE) over the wire FILL's region —
1M x 1500-B packets in 1536-B slots, every line read, one 128-B line per slot written back through —
beside the FILL and VERIFY of the same packets and the read-only probe, interleaved rounds, HIP events.
Picks the probe shape the bench line holds the FILL against. JSON lines.

  python tools/probe_rw_sweep.py
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import tcp_amd
    dev = torch.device("cuda:0")
    n, slot, tot = 1 << 20, 1536, 1500
    payload = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, payload.numel())
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = (np.arange(n, dtype=np.uint64) * 4096) % np.uint64(payload.numel() - 65536)
    segs["out_off"] = np.arange(n, dtype=np.uint64) * slot
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tot - 44, 17
    reg = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, tot - 20, reg, 0, None)
    doff = torch.from_numpy((np.arange(n, dtype=np.uint64) * slot).view(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    sta = torch.empty(n, dtype=torch.uint8, device=dev)
    pout = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    runs = {"fill": lambda: tcp_amd.ipv4_batch(reg, doff, n, slot, 0, out, sta),
            "verify": lambda: tcp_amd.ipv4_batch(reg, doff, n, slot, 1, out, sta)}
    # PROBE_GRIDS / PROBE_UNROLLS: comma lists (grid 0 = one tile per wave, XCD order; unroll 0 = C 4)
    grids = [int(x) for x in os.environ.get("PROBE_GRIDS", "512,2048,8192").split(",")]
    unrolls = [int(x) for x in os.environ.get("PROBE_UNROLLS", "1,2,4").split(",")]
    for mb in grids:
        for u in unrolls:
            for wr in (0, 1):
                t = (mb, u, 12 if wr else -1, tcp_amd.TUNE_PROBE_WRITE if wr else 0)
                runs[f"{'rw' if wr else 'rd'}_mb{mb}_u{u}"] = (lambda t=t: tcp_amd.stream_probe(reg, n * slot, pout, tune=t))
    times = {k: [] for k in runs}
    for _ in range(int(os.environ.get("ROUNDS", "3"))):
        for k, f in runs.items():
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                f()
            e1.record(st)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20)
    tcp_amd.ipv4_batch(reg, doff, n, slot, 1, out, sta)
    torch.cuda.synchronize()
    intact = bool((out == 0).all())   # the write-back probe left the packets as they were
    for k, ts in times.items():
        ms = statistics.median(ts)
        moved = n * slot + (n * 128 if k.startswith("rw") or k == "fill" else 0)
        print(json.dumps({"run": k, "ms_median": round(ms, 5), "ms_min": round(min(ts), 5),
                          "GB/s_moved": round(moved / (ms * 1e-3) / 1e9, 1), "packets_intact": intact}), flush=True)


if __name__ == "__main__":
    main()
