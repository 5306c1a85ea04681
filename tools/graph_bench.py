#!/usr/bin/env python3
"""Small-segment batches flushed one after another (1M x 64 B each, 16 distinct batches, 1 GiB
apart in HBM): per-batch time of (a) 16 eager launches, (b) the same 16 launches captured in one
HIP graph and replayed, (c) one tcpcsum_batch_uniform_multi_dev launch over the 16. HIP events on
the launch stream, interleaved rounds; every form's results compared with the eager ones.

  python tools/graph_bench.py [--rounds 5] [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--len", type=int, default=64)
    args = ap.parse_args()
    import torch
    import tcp_amd
    dev = torch.device("cuda:0")
    n, L, K = 1 << 20, args.len, 16
    bufs = []
    for j in range(K):
        d = torch.empty(n * L, dtype=torch.uint8, device=dev)
        tcp_amd.synth_fill(d, j * n * L, n * L)
        bufs.append(d)
    outs = {f: [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(K)] for f in ("eager", "graph", "multi")}

    def eager(o):
        for j in range(K):
            tcp_amd.batch_uniform(bufs[j], L, L, n, 0, out=o[j])

    arr = tcp_amd.ubatches([(bufs[j], L, L, n, 0, outs["multi"][j]) for j in range(K)])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        eager(outs["graph"])
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        eager(outs["graph"])
    forms = {"eager": lambda: eager(outs["eager"]), "graph": g.replay,
             "multi": lambda: tcp_amd.batch_uniform_multi(arr)}
    st = torch.cuda.current_stream()
    times = {f: [] for f in forms}
    for _ in range(args.rounds):
        for f, fn in forms.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            e1.record(st)
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(args.reps):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            times[f].append(e0.elapsed_time(e1) / args.reps / K)
    same = all(torch.equal(outs["eager"][j], outs[f][j]) for f in ("graph", "multi") for j in range(K))
    for f, t in times.items():
        ms = statistics.median(t)
        gbs = n * L / (ms * 1e-3) / 1e9
        print(json.dumps({"form": f, "batches": K, "segments": n, "len": L, "ms_per_batch_median": round(ms, 5),
                          "ms_per_batch_min": round(min(t), 5), "GB/s": round(gbs, 1),
                          "roofline_frac": round(gbs / 8000.0, 4), "same_results": same}), flush=True)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
