#!/usr/bin/env python3
"""Wire-kernel launch-shape sweep (tcpcsum_ipv4_batch_dev FILL and VERIFY), interleaved in one process
on bench.py's wire workload: 1M x 1500-B packets built by the fused builder in 1536-B slots. Every
variant's FILL must reproduce the builder's checks and its VERIFY must give 0. JSON lines.

  python tools/wire_sweep.py [--slot 1536] [--rounds 5] [--steps 20] blocks:unroll:shape ...

A variant "0:0:-1" is the built-in plan. WIRE_N: packets (default 1M)."""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slot", type=int, default=1536)
    ap.add_argument("--tot", type=int, default=1500)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--mix", action="store_true", help="bench.py's wire_mix workload (the flush mix) instead")
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    import numpy as np
    import torch
    import tcp_amd
    dev = torch.device("cuda:0")
    n, slot, tot = int(os.environ.get("WIRE_N", 1 << 20)), args.slot, args.tot
    tcp_len = tot - 20
    payload = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, payload.numel())
    if args.mix:
        import bench
        segs, region = bench.wire_mix_segments(n)
        slot = 1500   # the cap
    else:
        segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
        segs["payload_off"] = (np.arange(n, dtype=np.uint64) * 4096) % np.uint64(payload.numel() - 65536)
        segs["out_off"] = np.arange(n, dtype=np.uint64) * slot
        segs["saddr_be"] = 0x0100007F
        segs["daddr_be"] = np.arange(n, dtype=np.uint32)
        segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tcp_len - 24, 1 | 16
        region = n * slot
    reg = torch.zeros(region, dtype=torch.uint8, device=dev)
    built = torch.empty(n, dtype=torch.int16, device=dev)
    dsegs = torch.from_numpy(segs.view(np.uint8)).to(dev)
    tcp_amd.tx_build(payload, dsegs, n, 1456, reg, 0, built)
    del dsegs, payload
    doff = torch.from_numpy(segs["out_off"].astype(np.uint64).view(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    sta = torch.empty(n, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants]
    tunes = {v: tcp_amd.make_tuning(v[0], v[1], v[2], 0) for v in variants}
    modes = (("fill", tcp_amd.IPV4_FILL), ("verify", tcp_amd.IPV4_VERIFY))
    ok = {(v, m): True for v in variants for m, _ in modes}
    for v in variants:
        for name, mode in modes:
            tcp_amd.ipv4_batch(reg, doff, n, slot, mode, out, sta, tune=tunes[v])
            torch.cuda.synchronize()
            good = torch.equal(out, built) if name == "fill" else not bool(out.any().item())
            ok[(v, name)] = good and not bool(sta.any().item())
    times = {(v, m): [] for v in variants for m, _ in modes}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.rounds):
        for v in variants:
            for name, mode in modes:
                for _ in range(3):
                    tcp_amd.ipv4_batch(reg, doff, n, slot, mode, out, sta, tune=tunes[v])
                e0.record(st)
                for _ in range(args.steps):
                    tcp_amd.ipv4_batch(reg, doff, n, slot, mode, out, sta, tune=tunes[v])
                e1.record(st)
                torch.cuda.synchronize()
                times[(v, name)].append(e0.elapsed_time(e1) / args.steps)
    for (v, name), ts in times.items():
        print(json.dumps({"n": n, "workload": "flush_mix" if args.mix else f"slots{slot}", "max_blocks": v[0], "unroll": v[1], "shape": v[2], "mode": name,
                          "med_ms": round(statistics.median(ts), 5), "min_ms": round(min(ts), 5),
                          "ok": ok[(v, name)]}), flush=True)


if __name__ == "__main__":
    main()
