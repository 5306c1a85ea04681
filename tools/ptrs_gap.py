#!/usr/bin/env python3
"""Region vs pointer-per-packet wire batches on the same small packets.

Two device-resident workloads built by the fused builder (context.c:169-206
framing): 4M packed 84-B packets and 1M packed IMIX packets (7:4:1 of 64/576/
1500-B TCP segments). Each is checksummed (VERIFY) through
  region       tcpcsum_ipv4_batch_dev (one region + offsets), auto shape
  ptrs         tcpcsum_ipv4_batch_ptrs_dev (one address + length per packet), auto
               shape, no size hint (the shape is sized by cap: n x cap bytes)
  ptrs_hint    the same with bytes_hint = the summed lengths
  region_lb    region, forced balanced kernel (shape 8: k_ipv4_lb<4, PL=false>)
  ptrs_lb      pointers, forced balanced kernel (k_ipv4_lb<4, PL=true>)
interleaved over rounds, HIP events on the launch stream; results compared.
One JSON line per (workload, path).

  python tools/ptrs_gap.py [--rounds 5] [--only 84|imix]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    import tcp_amd
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    rng = np.random.default_rng(8)
    n = 1 << 20
    payload = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, payload.numel())

    def build(offs, tl, region_bytes):
        m = offs.size
        segs = np.zeros(m, tcp_amd.TXSEG_DTYPE)
        segs["out_off"] = offs
        segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(m, dtype=np.uint32)
        segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tl - 24, 1 | 16
        reg = torch.empty(region_bytes, dtype=torch.uint8, device=dev)
        tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), m, int(tl.max()), reg, 0, None)
        return reg

    works = []
    if args.only in ("", "84"):
        m = 1 << 22
        offs = np.arange(m, dtype=np.uint64) * 84
        works.append(("4Mx84_packed", build(offs, np.full(m, 64, np.uint32), m * 84), offs,
                      np.full(m, 84, np.uint32)))
    if args.only in ("", "imix"):
        tl = rng.choice(np.array([64, 576, 1500], np.uint32), n, p=[7 / 12, 4 / 12, 1 / 12])
        pl = (tl + 20).astype(np.uint64)
        offs = np.concatenate([[0], np.cumsum(pl)[:-1]]).astype(np.uint64)
        works.append(("1M_imix_packed", build(offs, tl, int(pl.sum())), offs, pl.astype(np.uint32)))
    torch.cuda.synchronize()
    for name, reg, offs, lens in works:
        m = offs.size
        doff = torch.from_numpy(offs.view(np.int64)).to(dev)
        dptr = doff + reg.data_ptr()
        dlen = torch.from_numpy(lens.view(np.int32)).to(dev)
        out = torch.empty(m, dtype=torch.int16, device=dev)
        sta = torch.empty(m, dtype=torch.uint8, device=dev)
        hint = int(lens.sum())
        lb = tcp_amd.make_tuning(0, 0, 8, 0)
        paths = {
            "region": lambda: tcp_amd.ipv4_batch(reg, doff, m, 1536, 1, out, sta),
            "ptrs": lambda: tcp_amd.ipv4_batch_ptrs(dptr, dlen, m, 1536, 1, out, sta),
            "ptrs_hint": lambda: tcp_amd.ipv4_batch_ptrs(dptr, dlen, m, 1536, 1, out, sta, bytes_hint=hint),
            "region_lb": lambda: tcp_amd.ipv4_batch(reg, doff, m, 1536, 1, out, sta, tune=lb),
            "ptrs_lb": lambda: tcp_amd.ipv4_batch_ptrs(dptr, dlen, m, 1536, 1, out, sta, tune=lb),
        }
        ref = None
        equal = True
        for k, f in paths.items():
            f()
            got = (out.clone(), sta.clone())
            if ref is None:
                ref = got
            equal = equal and torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])
        ok = bool((ref[0] == 0).all().item() and (ref[1] == 0).all().item())
        res = {k: [] for k in paths}
        for _ in range(args.rounds):
            for k, f in paths.items():
                for _ in range(3):
                    f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(20):
                    f()
                e1.record(st)
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) / 20)
        for k, ts in res.items():
            print(json.dumps({"measure": name, "path": k, "ms_median": round(statistics.median(ts), 4),
                              "ms_min": round(min(ts), 4), "results_equal": equal, "verify_all_zero": ok,
                              "packets": m, "tcp_bytes": int(lens.sum()) - 20 * m}), flush=True)


if __name__ == "__main__":
    main()
