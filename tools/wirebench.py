#!/usr/bin/env python3
"""Device-resident throughput of the ragged-descriptor and IPv4 wire kernels.

  * tcpcsum_batch_desc_dev on 1M segments with IMIX-like lengths
    (7:4:1 of 64 B, 576 B, 1500 B, random offsets in a 1.5 GB region);
  * tcpcsum_ipv4_batch_dev FILL and VERIFY on 1M IPv4/TCP packets of 1500 B
    in 1536-B slots (the reference's packets, device-resident).
Algorithmic bytes = the TCP segment bytes summed (+ the IP headers read for
the wire path, not counted). JSON lines.
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

    def timeit(fn, steps=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps * 1e-3

    rng = np.random.default_rng(0)
    n = 1 << 20
    region = 1536 * n
    data = torch.empty(region, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(data, 0, region)
    lens = rng.choice(np.array([64, 576, 1500], np.uint32), n, p=[7 / 12, 4 / 12, 1 / 12])
    desc = np.zeros(n, tcp_amd.DESC_DTYPE)
    desc["offset"] = np.arange(n, dtype=np.uint64) * 1536 + rng.integers(0, 8, n).astype(np.uint64) * 4
    desc["len"] = lens
    desc["sum_start"] = rng.integers(0, 393211, n, dtype=np.uint32)
    ddesc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    for sorted_ in (False, True):
        if sorted_:   # same segments, sorted by length (how a caller can bin a batch)
            order = np.argsort(lens, kind="stable")
            d2 = desc[order]
            ddesc = torch.from_numpy(d2.view(np.uint8)).to(dev)
        grid = ([(mb, un, sh) for sh in (-1, 2, 3) for mb in (2048, 8192) for un in (1, 2)]
                if "--sweep" in sys.argv else [(0, 0, -1), (0, 0, 7), (0, 0, 8), (2048, 0, 8)])
        for mb, un, sh in grid:
            tcp_amd.set_tuning(mb, un, sh, 0)
            t = timeit(lambda: tcp_amd.batch_desc(data, ddesc, n, 1500, out))
            print(json.dumps({"measure": "desc_imix_1M", "sorted_by_len": sorted_, "max_blocks": mb,
                              "unroll": un, "shape": sh,
                              "ms": round(t * 1e3, 4), "GB/s": round(int(lens.sum()) / t / 1e9, 1),
                              "Mseg/s": round(n / t / 1e6, 1)}), flush=True)
        tcp_amd.set_tuning(0, 0, -1, 0)

    # uniform-length descriptors: where the lane-group kernels are at home
    for L in (64, 1500):
        desc = np.zeros(n, tcp_amd.DESC_DTYPE)
        desc["offset"] = np.arange(n, dtype=np.uint64) * 1536 + rng.integers(0, 8, n).astype(np.uint64) * 4
        desc["len"] = L
        ddesc = torch.from_numpy(desc.view(np.uint8)).to(dev)
        for sh in (-1, 7, 8):
            tcp_amd.set_tuning(0, 0, sh, 0)
            t = timeit(lambda: tcp_amd.batch_desc(data, ddesc, n, L, out))
            print(json.dumps({"measure": f"desc_1Mx{L}", "shape": sh, "ms": round(t * 1e3, 4),
                              "GB/s": round(n * L / t / 1e9, 1), "Mseg/s": round(n / t / 1e6, 1)}), flush=True)
        tcp_amd.set_tuning(0, 0, -1, 0)

    # wire: 1M packets of 1500 B (IP 20 + TCP 24 + 1456 payload) in 1536-B slots
    payload = torch.empty(n * 1456, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, n * 1456)
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = np.arange(n, dtype=np.uint64) * 1456
    segs["out_off"] = np.arange(n, dtype=np.uint64) * 1536
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"] = 4000, 45001, 1456
    segs["flags"] = 1 | 16
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, 1456, data, 0, None)
    offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * 1536).view(np.int64)).to(dev)
    stat = torch.empty(n, dtype=torch.uint8, device=dev)
    for name, mode in (("FILL", tcp_amd.IPV4_FILL), ("VERIFY", tcp_amd.IPV4_VERIFY)):
        grid = ([(mb, un, sh) for sh in (-1, 3, 4) for mb in (2048, 8192) for un in (1, 2)]
                if "--sweep" in sys.argv else [(0, 0, -1), (0, 0, 8), (0, 0, 9)])
        for mb, un, sh in grid:
            tcp_amd.set_tuning(mb, un, sh, 0)
            t = timeit(lambda: tcp_amd.ipv4_batch(data, offs, n, 1536, mode, out, stat))
            print(json.dumps({"measure": "ipv4_1Mx1500", "mode": name, "max_blocks": mb, "unroll": un, "shape": sh,
                              "ms": round(t * 1e3, 4), "GB/s_tcp_bytes": round(n * 1480 / t / 1e9, 1),
                              "Mpkt/s": round(n / t / 1e6, 1)}), flush=True)
        tcp_amd.set_tuning(0, 0, -1, 0)
    ok = bool((out == 0).all().item()) and bool((stat == 0).all().item())
    print(json.dumps({"measure": "ipv4_verify_all_zero", "ok": ok}))

    # pure ACKs (44 B: IP 20 + TCP 24, no payload) in 1536-B slots
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = 0
    segs["out_off"] = np.arange(n, dtype=np.uint64) * 1536
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, 0, 16
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), n, 0, data, 0, None)
    for sh in (-1, 0, 8, 9):
        tcp_amd.set_tuning(0, 0, sh, 0)
        t = timeit(lambda: tcp_amd.ipv4_batch(data, offs, n, 1536, tcp_amd.IPV4_VERIFY, out, stat))
        ok = bool((out == 0).all().item()) and bool((stat == 0).all().item())
        print(json.dumps({"measure": "ipv4_1Mx44_ack_in_1536_slots_verify", "shape": sh, "ms": round(t * 1e3, 4),
                          "Mpkt/s": round(n / t / 1e6, 1), "ok": ok}), flush=True)
    tcp_amd.set_tuning(0, 0, -1, 0)

    # packed small packets (64-B TCP segments back to back, cap 1536): the next
    # offset bounds each packet's speculative span
    np_ = 1 << 22
    plen = 84   # IP 20 + TCP 24 + 40 payload
    segs = np.zeros(np_, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = 0
    segs["out_off"] = np.arange(np_, dtype=np.uint64) * plen
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(np_, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, 40, 1 | 16
    small = torch.empty(np_ * plen, dtype=torch.uint8, device=dev)
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), np_, 40, small, 0, None)
    soffs = torch.from_numpy((np.arange(np_, dtype=np.uint64) * plen).view(np.int64)).to(dev)
    sout = torch.empty(np_, dtype=torch.int16, device=dev)
    sst = torch.empty(np_, dtype=torch.uint8, device=dev)
    for sh in ((-1, 0, 6, 7, 5, 8, 9) if "--sweep" in sys.argv else (-1, 8, 9)):
        tcp_amd.set_tuning(0, 0, sh, 0)
        t = timeit(lambda: tcp_amd.ipv4_batch(small, soffs, np_, 1536, tcp_amd.IPV4_VERIFY, sout, sst))
        ok = bool((sout == 0).all().item()) and bool((sst == 0).all().item())
        print(json.dumps({"measure": "ipv4_4Mx84_packed_verify", "shape": sh, "ms": round(t * 1e3, 4),
                          "GB/s_packet_bytes": round(np_ * plen / t / 1e9, 1), "Mpkt/s": round(np_ / t / 1e6, 1),
                          "ok": ok}), flush=True)
    tcp_amd.set_tuning(0, 0, -1, 0)
    del small

    # packed IMIX (7:4:1 of 64, 576, 1500-byte TCP segments), back to back
    ni = 1 << 20
    tl = rng.choice(np.array([64, 576, 1500], np.uint32), ni, p=[7 / 12, 4 / 12, 1 / 12])
    plens = (tl + 20).astype(np.uint64)            # IP 20 + TCP (24-byte header + payload)
    ioff = np.concatenate([[0], np.cumsum(plens)[:-1]]).astype(np.uint64)
    segs = np.zeros(ni, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = 0
    segs["out_off"] = ioff
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(ni, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tl - 24, 1 | 16
    ireg = torch.empty(int(plens.sum()), dtype=torch.uint8, device=dev)
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), ni, 1500, ireg, 0, None)
    ioffs = torch.from_numpy(ioff.view(np.int64)).to(dev)
    iout = torch.empty(ni, dtype=torch.int16, device=dev)
    ist = torch.empty(ni, dtype=torch.uint8, device=dev)
    for sh in ((-1, 0, 6, 7, 5, 4, 8, 9) if "--sweep" in sys.argv else (-1, 8, 9)):
        for un in ((1, 2) if "--sweep" in sys.argv else (0,)):
            tcp_amd.set_tuning(0, un, sh, 0)
            t = timeit(lambda: tcp_amd.ipv4_batch(ireg, ioffs, ni, 1536, tcp_amd.IPV4_VERIFY, iout, ist))
            ok = bool((iout == 0).all().item()) and bool((ist == 0).all().item())
            print(json.dumps({"measure": "ipv4_1M_imix_packed_verify", "shape": sh, "unroll": un,
                              "ms": round(t * 1e3, 4), "GB/s_tcp_bytes": round(int(tl.sum()) / t / 1e9, 1),
                              "Mpkt/s": round(ni / t / 1e6, 1), "ok": ok}), flush=True)
    tcp_amd.set_tuning(0, 0, -1, 0)
    del ireg

    # jumbo: 128K packets of 9000 B in 9216-B slots
    nj, jl, js = 1 << 17, 8956, 9216
    jpay = torch.empty(nj * jl, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(jpay, 7, nj * jl)
    segs = np.zeros(nj, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = np.arange(nj, dtype=np.uint64) * jl
    segs["out_off"] = np.arange(nj, dtype=np.uint64) * js
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(nj, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, jl, 1 | 16
    jreg = torch.empty(nj * js, dtype=torch.uint8, device=dev)
    tcp_amd.tx_build(jpay, torch.from_numpy(segs.view(np.uint8)).to(dev), nj, jl, jreg, 0, None)
    del jpay
    joffs = torch.from_numpy((np.arange(nj, dtype=np.uint64) * js).view(np.int64)).to(dev)
    jout = torch.empty(nj, dtype=torch.int16, device=dev)
    jst = torch.empty(nj, dtype=torch.uint8, device=dev)
    grid = ([(mb, un, sh) for sh in (-1, 1, 2, 4, 5) for mb in (2048, 8192) for un in (1, 2)]
            if "--sweep" in sys.argv else [(0, 0, -1), (0, 0, 9)])
    for mb, un, sh in grid:
        tcp_amd.set_tuning(mb, un, sh, 0)
        t = timeit(lambda: tcp_amd.ipv4_batch(jreg, joffs, nj, js, tcp_amd.IPV4_VERIFY, jout, jst))
        print(json.dumps({"measure": "ipv4_128Kx9000_verify", "max_blocks": mb, "unroll": un, "shape": sh,
                          "ms": round(t * 1e3, 4), "GB/s_tcp_bytes": round(nj * 8980 / t / 1e9, 1)}), flush=True)
    tcp_amd.set_tuning(0, 0, -1, 0)
    ok = bool((jout == 0).all().item()) and bool((jst == 0).all().item())
    print(json.dumps({"measure": "ipv4_jumbo_verify_all_zero", "ok": ok}))


if __name__ == "__main__":
    main()
