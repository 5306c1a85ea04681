#!/usr/bin/env python3
"""Launch-shape sweep for the uniform checksum kernel (interleaved rounds, one process).

  python tools/sweep.py [--config 1500] [--rounds 5] [--steps 50]

Prints one line per (max_blocks, unroll) variant: median and min kernel ms over
rounds, GB/s of algorithmic bytes. Variants are interleaved within each round
(cdna_hip_programming.md §5.4 rule 24).
"""
import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1500")
    ap.add_argument("--len", type=int, default=0, help="custom segment length (total ~1.5 GB)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--blocks", default="256,512,1024,2048,4096,8192,0")
    ap.add_argument("--unrolls", default="1,2,4")
    ap.add_argument("--shapes", default="-1")
    ap.add_argument("--flags", default="0", help="TCPCSUM_TUNE_* bits: 1 pipe on, 2 pipe off, 4 nt on, 8 nt off")
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--rot", type=int, default=0, help="rotating input buffers (0: enough for >= 1 GiB in total)")
    ap.add_argument("--probe-shapes", default="0:0:-1", help="probe max_blocks:unroll:shape triples, with --probe")
    args = ap.parse_args()
    import torch
    import tcp_amd
    from bench import CONFIGS
    if args.len:
        L = args.len
        per = (1572864000 // L)
        args.config = f"len{L}"
    else:
        per, L, _ = CONFIGS[args.config]
    nbytes = per * L
    rot = max(1, math.ceil((1 << 30) / nbytes)) if nbytes < (1 << 30) else 1
    if args.rot:
        rot = args.rot
    dev = torch.device("cuda:0")
    bufs, sss = [], []
    for r in range(rot):
        d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        tcp_amd.synth_fill(d, r * nbytes, nbytes)
        s = torch.empty(per, dtype=torch.int32, device=dev)
        tcp_amd.synth_pseudo(s, 0, per, L)
        bufs.append(d)
        sss.append(s)
    out = torch.empty(per, dtype=torch.int16, device=dev)
    # every variant's results of rotation 0 must equal the built-in plan's
    tcp_amd.set_tuning(0, 0, -1, 0)
    tcp_amd.batch_uniform(bufs[0], L, L, per, sss[0], out=out)
    want = out.clone()
    variants = []
    for fl in [int(x) for x in args.flags.split(",")]:
        for sh in [int(x) for x in args.shapes.split(",")]:
            for b in [int(x) for x in args.blocks.split(",")]:
                for u in [int(x) for x in args.unrolls.split(",")]:
                    variants.append((b, u, sh, fl))
    times = {v: [] for v in variants}
    same = {}
    ptimes = {}
    pshapes = [tuple(int(y) for y in (x + ":-1").split(":")[:3]) for x in args.probe_shapes.split(",")]
    st = torch.cuda.current_stream()
    for rnd in range(args.rounds):
        for v in variants:
            tcp_amd.set_tuning(*v)
            for i in range(3):
                tcp_amd.batch_uniform(bufs[i % rot], L, L, per, sss[i % rot], out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(args.steps):
                tcp_amd.batch_uniform(bufs[i % rot], L, L, per, sss[i % rot], out=out)
            e1.record(st)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.steps)
            out.zero_()
            tcp_amd.batch_uniform(bufs[0], L, L, per, sss[0], out=out)
            same[v] = same.get(v, True) and bool(torch.equal(out, want))
        if args.probe:
            po = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=dev)
            for ps in pshapes:
                tcp_amd.set_tuning(ps[0], ps[1], ps[2], 0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for i in range(args.steps):
                    tcp_amd.stream_probe(bufs[i % rot], (nbytes // 16) * 16, po)
                e1.record(st)
                torch.cuda.synchronize()
                ptimes.setdefault(ps, []).append(e0.elapsed_time(e1) / args.steps)
    tcp_amd.set_tuning(0, 0, -1, 0)
    res = []
    for v in variants:
        med, mn = statistics.median(times[v]), min(times[v])
        res.append({"max_blocks": v[0], "unroll": v[1], "shape": v[2], "flags": v[3], "med_ms": round(med, 5), "min_ms": round(mn, 5),
                    "GB/s_med": round(nbytes / med / 1e6, 1), "GB/s_best": round(nbytes / mn / 1e6, 1),
                    "same_results": same[v]})
        print(json.dumps({"config": args.config, **res[-1]}), flush=True)
    for ps, ts in ptimes.items():
        med = statistics.median(ts)
        print(json.dumps({"config": args.config, "probe_max_blocks": ps[0], "probe_unroll": ps[1], "probe_shape": ps[2],
                          "probe_med_ms": round(med, 5), "probe_GB/s": round(nbytes / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
