#!/usr/bin/env python3
"""Launch-shape sweep of tcpcsum_batch_uniform_multi_dev on small uniform segments.

BASELINE's 64-B config (1M x 64 B per batch, SURVEY.md Appendix B stream) in
rotating batches (>= 2 GiB in all, so no launch reads bytes the Infinity Cache
still holds); each point launches K batches at a time and reports the kernel
time per batch (HIP events on the launch stream), interleaved over rounds so
box drift hits every point alike. One JSON line per point and round.

  python tools/multi_sweep.py [--len 64] [--rounds 3] [--steps 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=64)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ks", default="1,4,8,16")
    ap.add_argument("--unrolls", default="4,8")
    ap.add_argument("--grids", default="0,8192,32768")
    ap.add_argument("--shapes", default="-1", help="forced lane-group shapes (-1 = auto)")
    args = ap.parse_args()
    import torch
    import tcp_amd
    dev = torch.device("cuda:0")
    L, n = args.len, args.n
    R = max(32, (2 << 30) // (n * L))
    bufs, sss, outs = [], [], []
    for r in range(R):
        d = torch.empty(n * L, dtype=torch.uint8, device=dev)
        tcp_amd.synth_fill(d, r * n * L, n * L)
        s = torch.empty(n, dtype=torch.int32, device=dev)
        tcp_amd.synth_pseudo(s, 0, n, L)
        bufs.append(d)
        sss.append(s)
    outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(16)]
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    points = [(k, u, g, sh) for k in map(int, args.ks.split(",")) for u in map(int, args.unrolls.split(","))
              for g in map(int, args.grids.split(",")) for sh in map(int, args.shapes.split(","))]
    for rnd in range(args.rounds):
        for K, unroll, grid, shape in points:
            groups = [tcp_amd.ubatches([(bufs[(g * K + j) % R], L, L, n, sss[(g * K + j) % R], outs[j])
                                        for j in range(K)]) for g in range(R // K)]
            tune = tcp_amd.make_tuning(grid, unroll, shape, 0)
            for i in range(3):
                tcp_amd.batch_uniform_multi(groups[i % len(groups)], tune=tune)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(args.steps):
                tcp_amd.batch_uniform_multi(groups[i % len(groups)], tune=tune)
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            per = ms / K
            gbs = n * L / (per * 1e-3) / 1e9
            print(json.dumps({"round": rnd, "len": L, "n": n, "K": K, "unroll": unroll, "max_blocks": grid, "shape": shape,
                              "ms_per_launch": round(ms, 5), "ms_per_batch": round(per, 5),
                              "GB/s": round(gbs, 1), "frac": round(gbs / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
