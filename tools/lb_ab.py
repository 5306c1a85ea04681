#!/usr/bin/env python3
"""A/B of the balanced chunk-space kernels (k_desc_lb, k_ipv4_lb) against a
previous build, interleaved in one process (HIP events on the launch stream).

Workloads (device-resident, as tools/wirebench.py builds them):
  * ragged descriptors: 1M IMIX segments (7:4:1 of 64/576/1500 B, 4-B aligned
    offsets in 1536-B slots), 1M x 1500 B and 1M x 64 B — forced balanced (shape 7);
  * wire VERIFY: 1M packed IMIX packets, 4M packed 84-B packets, 1M pure ACKs in
    1536-B slots — forced balanced (shape 8).
Results must agree between the two builds. JSON lines.

  python tools/lb_ab.py [old.so]     (round-1 ABI or ABI v2 builds; LB_ONLY=name runs one workload)
"""
import ctypes
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

    old_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tcp_amd", "ab", "libtcpcsum_r01.so")
    new = tcp_amd.lib()
    old = ctypes.CDLL(old_path)
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    v2 = hasattr(old, "tcpcsum_tuning_check")   # ABI v2: per-call tuning (an earlier round-2 build)
    if v2:
        old.tcpcsum_ipv4_batch_dev.argtypes = [vp, u64, vp, u64, u32, ctypes.c_int, vp, vp, vp, vp]
        old.tcpcsum_batch_desc_dev.argtypes = [vp, vp, u64, u32, vp, vp, vp]
    else:
        old.tcpcsum_ipv4_batch_dev.argtypes = [vp, u64, vp, u64, u32, ctypes.c_int, vp, vp, vp]
        old.tcpcsum_batch_desc_dev.argtypes = [vp, vp, u64, u32, vp, vp]
        old.tcpcsum_set_tuning.argtypes = [ctypes.c_int] * 4
    old_tag = os.path.basename(old_path).replace("libtcpcsum_", "").replace(".so", "")
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    h = st.cuda_stream
    rng = np.random.default_rng(0)

    def timeit(fn, steps=30):
        for _ in range(3):
            assert fn() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    only = os.environ.get("LB_ONLY")   # run just this workload (profiling)

    def ab(name, f_old, f_new, out, nbytes, rounds=7):
        if only and only != name:
            return
        f_old()
        a = out.clone()
        f_new()
        same = bool(torch.equal(a, out))
        res = {old_tag: [], "head": []}
        for _ in range(rounds):
            res[old_tag].append(timeit(f_old))
            res["head"].append(timeit(f_new))
        for lib, ts in res.items():
            ms = statistics.median(ts)
            print(json.dumps({"measure": name, "lib": lib, "ms_median": round(ms, 4), "ms_min": round(min(ts), 4),
                              "GB/s": round(nbytes / (ms * 1e-3) / 1e9, 1), "results_equal": same}), flush=True)

    n = 1 << 20
    data = torch.empty(1536 * n, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(data, 0, 1536 * n)
    out = torch.empty(1 << 22, dtype=torch.int16, device=dev)
    sta = torch.empty(1 << 22, dtype=torch.uint8, device=dev)
    t7 = tcp_amd.Tuning(0, 0, 7, 0)
    t8 = tcp_amd.Tuning(0, 0, 8, 0)
    # LB_HEAD_DESC / LB_HEAD_WIRE="max_blocks,unroll,shape,flags": the head build's launch (the old build keeps 7 / 8)
    h7 = tcp_amd.Tuning(*map(int, os.environ["LB_HEAD_DESC"].split(","))) if "LB_HEAD_DESC" in os.environ else t7
    h8 = tcp_amd.Tuning(*map(int, os.environ["LB_HEAD_WIRE"].split(","))) if "LB_HEAD_WIRE" in os.environ else t8

    for name, lens in (("desc_lb_1M_imix", rng.choice(np.array([64, 576, 1500], np.uint32), n,
                                                       p=[7 / 12, 4 / 12, 1 / 12])),
                       ("desc_lb_1Mx1500", np.full(n, 1500, np.uint32)),
                       ("desc_lb_1Mx64", np.full(n, 64, np.uint32))):
        desc = np.zeros(n, tcp_amd.DESC_DTYPE)
        desc["offset"] = np.arange(n, dtype=np.uint64) * 1536 + rng.integers(0, 8, n).astype(np.uint64) * 4
        desc["len"] = lens
        desc["sum_start"] = rng.integers(0, 393211, n, dtype=np.uint32)
        dd = torch.from_numpy(desc.view(np.uint8)).to(dev)
        mx = int(lens.max())

        def f_old():
            if v2:
                return old.tcpcsum_batch_desc_dev(data.data_ptr(), dd.data_ptr(), n, mx, out.data_ptr(), h,
                                                  ctypes.byref(t7))
            old.tcpcsum_set_tuning(0, 0, 7, 0)
            return old.tcpcsum_batch_desc_dev(data.data_ptr(), dd.data_ptr(), n, mx, out.data_ptr(), h)

        def f_new():
            return new.tcpcsum_batch_desc_dev(data.data_ptr(), dd.data_ptr(), n, mx, out.data_ptr(), h,
                                              ctypes.byref(h7))
        ab(name, f_old, f_new, out[:n], int(lens.sum()))

    # wire workloads, built on device by the fused builder (context.c:169-206 framing)
    def build(offs, tl, region_bytes):
        m = offs.size
        segs = np.zeros(m, tcp_amd.TXSEG_DTYPE)
        segs["out_off"] = offs
        segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(m, dtype=np.uint32)
        segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tl - 24, 1 | 16
        reg = torch.empty(region_bytes, dtype=torch.uint8, device=dev)
        tcp_amd.tx_build(data, torch.from_numpy(segs.view(np.uint8)).to(dev), m, int(tl.max()), reg, 0, None)
        return reg, torch.from_numpy(offs.view(np.int64)).to(dev)

    tl = rng.choice(np.array([64, 576, 1500], np.uint32), n, p=[7 / 12, 4 / 12, 1 / 12])
    pl = (tl + 20).astype(np.uint64)
    io = np.concatenate([[0], np.cumsum(pl)[:-1]]).astype(np.uint64)
    w_imix = build(io, tl, int(pl.sum())) + (n, int(tl.sum()))
    m84 = 1 << 22
    w_84 = build(np.arange(m84, dtype=np.uint64) * 84, np.full(m84, 64, np.uint32), m84 * 84) + (m84, m84 * 64)
    w_ack = build(np.arange(n, dtype=np.uint64) * 1536, np.full(n, 24, np.uint32), n * 1536) + (n, n * 24)
    for name, (reg, offs, m, nbytes) in (("ipv4_lb_1M_imix_packed_verify", w_imix),
                                         ("ipv4_lb_4Mx84_packed_verify", w_84),
                                         ("ipv4_lb_1M_ack_slots1536_verify", w_ack)):
        R = reg.numel()

        def f_old():
            if v2:
                return old.tcpcsum_ipv4_batch_dev(reg.data_ptr(), R, offs.data_ptr(), m, 1536, 1, out.data_ptr(),
                                                  sta.data_ptr(), h, ctypes.byref(t8))
            old.tcpcsum_set_tuning(0, 0, 8, 0)
            return old.tcpcsum_ipv4_batch_dev(reg.data_ptr(), R, offs.data_ptr(), m, 1536, 1, out.data_ptr(),
                                              sta.data_ptr(), h)

        def f_new():
            return new.tcpcsum_ipv4_batch_dev(reg.data_ptr(), R, offs.data_ptr(), m, 1536, 1, out.data_ptr(),
                                              sta.data_ptr(), h, ctypes.byref(h8))
        ab(name, f_old, f_new, out[:m], nbytes)
        if only and only != name:
            continue
        ok = bool((out[:m] == 0).all().item()) and bool((sta[:m] == 0).all().item())
        print(json.dumps({"measure": name, "verify_all_zero": ok}), flush=True)
    if not v2:
        old.tcpcsum_set_tuning(0, 0, -1, 0)


if __name__ == "__main__":
    main()
