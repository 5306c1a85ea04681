#!/usr/bin/env python3
"""Launch-shape sweep of the lane-group wire kernel (k_ipv4) on 1M IPv4/TCP
packets of 1500 B in 1536-B slots (SLOT / PAYLOAD env: other sizes),
device-resident, VERIFY and FILL; SHAPES / BLOCKS / UNROLLS env: the grid.

Rounds are interleaved (every configuration once per round, median over
rounds) so box-level drift affects all shapes alike. JSON lines.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import tcp_amd

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    n, slot = int(os.environ.get("N", str(1 << 20))), int(os.environ.get("SLOT", "1536"))
    pay = int(os.environ.get("PAYLOAD", str(slot - 80)))   # TCP payload bytes (packet = pay + 44)
    payload = torch.empty(n * pay, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, n * pay)
    data = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = np.arange(n, dtype=np.uint64) * pay
    segs["out_off"] = np.arange(n, dtype=np.uint64) * slot
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, pay, 1 | 16
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, pay, data, 0, None)
    offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * slot).view(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    stat = torch.empty(n, dtype=torch.uint8, device=dev)
    shapes = [int(x) for x in os.environ.get("SHAPES", "-1,1,3,4,5,7").split(",")]
    blocks = [int(x) for x in os.environ.get("BLOCKS", "0,512,1024,2048,4096").split(",")]
    unrolls = [int(x) for x in os.environ.get("UNROLLS", "1,2").split(",")]
    flags = [int(x) for x in os.environ.get("FLAGS", "0").split(",")]   # TCPCSUM_TUNE_* bits
    cfgs = [(m, sh, mb, un, fl) for m in ("VERIFY", "FILL") for sh in shapes for mb in blocks for un in unrolls
            for fl in flags]
    res = {c: [] for c in cfgs}
    checked = {}
    for rnd in range(5):
        for c in cfgs:
            m, sh, mb, un, fl = c
            tcp_amd.set_tuning(mb, un, sh, fl)
            mode = tcp_amd.IPV4_VERIFY if m == "VERIFY" else tcp_amd.IPV4_FILL
            fn = lambda: tcp_amd.ipv4_batch(data, offs, n, slot, mode, out, stat)
            fn()
            if rnd == 0:
                # this configuration's own result: VERIFY must give all zeros; FILL must leave
                # checks that verify to zero (checked with the default shape)
                if m == "FILL":
                    tcp_amd.set_tuning(0, 0, -1, 0)
                    tcp_amd.ipv4_batch(data, offs, n, slot, tcp_amd.IPV4_VERIFY, out, stat)
                    tcp_amd.set_tuning(mb, un, sh, fl)
                checked[c] = bool((out == 0).all().item()) and bool((stat == 0).all().item())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(10):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            res[c].append(e0.elapsed_time(e1) / 10)
        tcp_amd.set_tuning(0, 0, -1, 0)
        print(json.dumps({"round": rnd}), flush=True)
    for c, ts in sorted(res.items(), key=lambda kv: (kv[0][0], sorted(kv[1])[2])):
        m, sh, mb, un, fl = c
        ms = sorted(ts)[len(ts) // 2]
        print(json.dumps({"measure": f"ipv4_shape_sweep_1Mx{pay + 44}_slots{slot}", "mode": m, "shape": sh,
                          "max_blocks": mb, "unroll": un, "flags": fl, "ms": round(ms, 4),
                          "GB/s_tcp_bytes": round(n * (pay + 24) / (ms * 1e-3) / 1e9, 1),
                          "verify_ok": checked[c]}), flush=True)


if __name__ == "__main__":
    main()
