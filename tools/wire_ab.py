#!/usr/bin/env python3
"""A/B of the wire kernel against a previous build, interleaved in one process.

Loads the current libtcpcsum.so and a previous build (default
tcp_amd/ab/libtcpcsum_r01.so: round 1, before the per-packet bound `plen` was
added to k_ipv4 / k_ipv4_lb) and times tcpcsum_ipv4_batch_dev FILL and VERIFY on
1M x 1500-B packets in 1536-B slots, device-resident, alternating the two
libraries round by round (HIP events on the launch stream). Also times the
current library's scatter-gather entry point (tcpcsum_ipv4_batch_ptrs_dev) on
the same packets addressed by pointer. JSON lines.

  python tools/wire_ab.py [old.so]
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
    from tests.packets import ip_packet

    old_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tcp_amd", "ab", "libtcpcsum_r01.so")
    new = tcp_amd.lib()
    old = ctypes.CDLL(old_path)
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    old.tcpcsum_ipv4_batch_dev.argtypes = [vp, u64, vp, u64, u32, ctypes.c_int, vp, vp, vp]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    n, slot = 1 << 20, 1536
    rng = np.random.default_rng(0)
    pk = np.frombuffer(ip_packet(rng, 1456), np.uint8)
    host = np.zeros(slot, np.uint8)
    host[:pk.size] = pk
    one = torch.from_numpy(host).to(dev)
    region = one.repeat(n)
    payload = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, n * slot)
    region.view(n, slot)[:, 44:1500] = payload.view(n, slot)[:, 44:1500]   # distinct payloads
    off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    ptrs = off + region.data_ptr()
    lens = torch.full((n,), 1500, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    sta = torch.empty(n, dtype=torch.uint8, device=dev)
    h = st.cuda_stream
    R = region.numel()

    def f_old(mode):
        return lambda: old.tcpcsum_ipv4_batch_dev(region.data_ptr(), R, off.data_ptr(), n, 1536, mode,
                                                  out.data_ptr(), sta.data_ptr(), h)

    def f_new(mode):
        return lambda: new.tcpcsum_ipv4_batch_dev(region.data_ptr(), R, off.data_ptr(), n, 1536, mode,
                                                  out.data_ptr(), sta.data_ptr(), h, None)

    def f_ptrs(mode):
        return lambda: new.tcpcsum_ipv4_batch_ptrs_dev(ptrs.data_ptr(), lens.data_ptr(), n, 1536, 0, mode,
                                                       out.data_ptr(), sta.data_ptr(), h, None)

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

    # results agree between the libraries
    checks = {}
    for mode in (0, 1):
        f_old(mode)()
        a = out.clone()
        f_new(mode)()
        b = out.clone()
        f_ptrs(mode)()
        c = out.clone()
        checks[mode] = bool(torch.equal(a, b) and torch.equal(b, c))
    dw = tcp_amd.Tuning(0, 0, -1, tcp_amd.api.TUNE_FILL_DWORD)

    def f_dw(mode):
        return lambda: new.tcpcsum_ipv4_batch_dev(region.data_ptr(), R, off.data_ptr(), n, 1536, mode,
                                                  out.data_ptr(), sta.data_ptr(), h, ctypes.byref(dw))
    f_new(0)()
    ref_out, ref_reg = out.clone(), region.clone()
    f_dw(0)()
    checks["dw"] = bool(torch.equal(out, ref_out) and torch.equal(region, ref_reg))
    del ref_reg
    res = {}
    for rnd in range(7):
        for mode, mname in ((0, "FILL"), (1, "VERIFY")):
            libs = (("r01", f_old), ("head", f_new), ("head_ptrs", f_ptrs)) + ((("head_fill_dword", f_dw),)
                                                                                if mode == 0 else ())
            for lname, fn in libs:
                res.setdefault((mname, lname), []).append(timeit(fn(mode)))
    for (mname, lname), ts in sorted(res.items()):
        print(json.dumps({"measure": "wire_ab_1Mx1500_slots1536", "mode": mname, "lib": lname,
                          "ms_median": round(statistics.median(ts), 4), "ms_min": round(min(ts), 4),
                          "rounds": len(ts), "results_equal_across_libs": checks[0 if mname == "FILL" else 1],
                          "fill_dword_equal": checks["dw"]}),
              flush=True)

    # jumbo frames: 128K x 9000-B packets in 9216-B slots (the multi-round path)
    del region, payload, ptrs
    torch.cuda.empty_cache()
    nj, sj = 128 << 10, 9216
    pk = np.frombuffer(ip_packet(rng, 8956), np.uint8)
    host = np.zeros(sj, np.uint8)
    host[:pk.size] = pk
    jreg = torch.from_numpy(host).to(dev).repeat(nj)
    jpay = torch.empty(nj * sj, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(jpay, 0, nj * sj)
    jreg.view(nj, sj)[:, 44:9000] = jpay.view(nj, sj)[:, 44:9000]
    del jpay
    joff = torch.arange(nj, dtype=torch.int64, device=dev) * sj
    jout = torch.empty(nj, dtype=torch.int16, device=dev)
    jst = torch.empty(nj, dtype=torch.uint8, device=dev)
    JR = jreg.numel()

    def j_old(mode):
        return lambda: old.tcpcsum_ipv4_batch_dev(jreg.data_ptr(), JR, joff.data_ptr(), nj, 9216, mode,
                                                  jout.data_ptr(), jst.data_ptr(), h)

    def j_new(mode):
        return lambda: new.tcpcsum_ipv4_batch_dev(jreg.data_ptr(), JR, joff.data_ptr(), nj, 9216, mode,
                                                  jout.data_ptr(), jst.data_ptr(), h, None)
    jchk = {}
    for mode in (0, 1):
        j_old(mode)()
        a2 = jout.clone()
        j_new(mode)()
        jchk[mode] = bool(torch.equal(a2, jout))
    jres = {}
    for rnd in range(5):
        for mode, mname in ((0, "FILL"), (1, "VERIFY")):
            for lname, fn in (("r01", j_old), ("head", j_new)):
                jres.setdefault((mname, lname), []).append(timeit(fn(mode), 20))
    for (mname, lname), ts in sorted(jres.items()):
        print(json.dumps({"measure": "wire_ab_128Kx9000_slots9216", "mode": mname, "lib": lname,
                          "ms_median": round(statistics.median(ts), 4), "ms_min": round(min(ts), 4),
                          "GB/s_tcp_bytes": round(nj * 8980 / (statistics.median(ts) * 1e-3) / 1e9, 1),
                          "rounds": len(ts), "results_equal_across_libs": jchk[0 if mname == "FILL" else 1]}),
              flush=True)


if __name__ == "__main__":
    main()
