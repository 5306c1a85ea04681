#!/usr/bin/env python3
"""Sweep the read-only stream probe (k_probe) over launch shapes: the practical
HBM read ceiling for a 16-B-per-lane streaming access on this device.

  python tools/probe_sweep.py [--mib 1500] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1572864000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    import torch
    import tcp_amd
    nb = args.bytes // 16 * 16
    buf = torch.empty(nb, dtype=torch.uint8, device="cuda")
    tcp_amd.synth_fill(buf, 0, nb)
    parts = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    variants = [(b, u) for b in (256, 512, 1024, 2048, 4096, 8192) for u in (1, 2, 4)]
    times = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            tcp_amd.set_tuning(v[0], v[1], -1, 0)
            for _ in range(3):
                tcp_amd.stream_probe(buf, nb, parts)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.steps):
                tcp_amd.stream_probe(buf, nb, parts)
            e1.record(st)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.steps)
    tcp_amd.set_tuning(0, 0, -1, 0)
    for v in variants:
        med = statistics.median(times[v])
        print(json.dumps({"probe_blocks": v[0], "chunks_per_lane": 8 * v[1], "med_ms": round(med, 5),
                          "GB/s": round(nb / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
