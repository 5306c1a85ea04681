#!/usr/bin/env python3
"""Wire FILL store A/B: the check stored as one native u16
(context.c:208, TCPCSUM_TUNE_FILL_U16) vs the check's whole 128-B line written
through (sc0 sc1; the default where the line lies inside the packet), beside
VERIFY on the same packets. Exit 1 if the two FILLs ever differ.

Workloads (device-resident, built by the fused builder, context.c:169-206
framing): 1M x 1500-B packets in 1536-B slots; 1M packed 1500-B packets (only
packets whose check line lies inside them take the line store); 128K x 9000-B
jumbo packets in 9216-B slots. Interleaved rounds, HIP events on the launch
stream; FILL results and regions compared between the variants.

  python tools/fill_line_ab.py [--rounds 5]
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
    args = ap.parse_args()
    import numpy as np
    import torch
    import tcp_amd
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    payload = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, payload.numel())

    def build(offs, tl, region_bytes):
        m = offs.size
        segs = np.zeros(m, tcp_amd.TXSEG_DTYPE)
        segs["payload_off"] = (np.arange(m, dtype=np.uint64) * 4096) % np.uint64(payload.numel() - 65536)
        segs["out_off"] = offs
        segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(m, dtype=np.uint32)
        segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tl - 24, 1 | 16
        reg = torch.zeros(region_bytes, dtype=torch.uint8, device=dev)
        tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), m, int(tl.max()), reg, 0, None)
        return reg

    n = 1 << 20
    all_equal = True
    works = [("1Mx1500_slots1536", np.arange(n, dtype=np.uint64) * 1536, np.full(n, 1480, np.uint32), n * 1536, 1536),
             ("1Mx1500_packed", np.arange(n, dtype=np.uint64) * 1500, np.full(n, 1480, np.uint32), n * 1500, 1536),
             ("128Kx9000_slots9216", np.arange(n // 8, dtype=np.uint64) * 9216, np.full(n // 8, 8980, np.uint32),
              (n // 8) * 9216, 9216)]
    for name, offs, tl, rb, cap in works:
        reg = build(offs, tl, rb)
        m = offs.size
        doff = torch.from_numpy(offs.view(np.int64)).to(dev)
        out = torch.empty(m, dtype=torch.int16, device=dev)
        sta = torch.empty(m, dtype=torch.uint8, device=dev)
        u16 = tcp_amd.make_tuning(0, 0, -1, tcp_amd.TUNE_FILL_U16)
        half = tcp_amd.make_tuning(0, 0, -1, tcp_amd.TUNE_FILL_HALF)
        paths = {"fill_u16": lambda: tcp_amd.ipv4_batch(reg, doff, m, cap, 0, out, sta, tune=u16),
                 "fill_line": lambda: tcp_amd.ipv4_batch(reg, doff, m, cap, 0, out, sta),
                 "fill_half": lambda: tcp_amd.ipv4_batch(reg, doff, m, cap, 0, out, sta, tune=half),
                 "verify": lambda: tcp_amd.ipv4_batch(reg, doff, m, cap, 1, out, sta)}
        paths["fill_u16"]()
        a = (out.clone(), reg.clone())
        paths["fill_line"]()
        equal = bool(torch.equal(a[0], out) and torch.equal(a[1], reg))
        paths["fill_half"]()
        equal = equal and bool(torch.equal(a[0], out) and torch.equal(a[1], reg))
        if not equal:   # where the variants differ (bytes of the region, and results)
            d = (a[1] != reg).nonzero().flatten()
            dd = d.cpu().numpy()[:20]
            print(json.dumps({"measure": name, "region_diffs": int(d.numel()), "first": [int(x) for x in dd],
                              "slot_offsets": sorted({int(x) % cap for x in dd}),
                              "out_diffs": int((a[0] != out).sum().item())}), flush=True)
        del a
        paths["verify"]()
        ok = bool((out == 0).all().item() and (sta == 0).all().item())
        all_equal = all_equal and equal and ok
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
                              "ms_min": round(min(ts), 4), "fill_variants_equal": equal, "verify_all_zero": ok}),
                  flush=True)
        del reg
        torch.cuda.empty_cache()
    return 0 if all_equal else 1


if __name__ == "__main__":
    sys.exit(main())
