#!/usr/bin/env python3
"""Wire kernel (tcpcsum_ipv4_batch_dev) A/B: the in-tree library against ABI-v3
builds in tcp_amd/ab/, interleaved in one process on the same packets (built by
the fused builder, context.c:169-206 framing), HIP events on the launch stream.
VERIFY and FILL per workload; every build's FILL results and region must equal
the in-tree build's (`same`). JSON lines.

  python tools/wire_lib_ab.py [lib.so ...]   (default: tcp_amd/ab/libtcpcsum_wire*.so)
"""
import ctypes
import glob
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

    paths = sys.argv[1:] or sorted(glob.glob(os.path.join(REPO, "tcp_amd", "ab", "libtcpcsum_wire*.so")))
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    libs = {"in_tree": tcp_amd.lib()}
    for p in paths:
        lib = ctypes.CDLL(p)
        lib.tcpcsum_ipv4_batch_dev.argtypes = [vp, u64, vp, u64, u32, ctypes.c_int, vp, vp, vp, vp]
        lib.tcpcsum_ipv4_batch_dev.restype = ctypes.c_int
        libs[os.path.basename(p).replace("libtcpcsum_", "").replace(".so", "")] = lib
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    h = st.cuda_stream
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
    works = [("1Mx1500_slots1536", np.arange(n, dtype=np.uint64) * 1536, np.full(n, 1480, np.uint32), n * 1536, 1536),
             ("1Mx988_slots1024", np.arange(n, dtype=np.uint64) * 1024, np.full(n, 968, np.uint32), n * 1024, 1024),
             ("1Mx2000_slots2048", np.arange(n, dtype=np.uint64) * 2048, np.full(n, 1980, np.uint32), n * 2048, 2048),
             ("1Mx1500_packed", np.arange(n, dtype=np.uint64) * 1500, np.full(n, 1480, np.uint32), n * 1500, 1536),
             ("128Kx9000_slots9216", np.arange(n // 8, dtype=np.uint64) * 9216, np.full(n // 8, 8980, np.uint32),
              (n // 8) * 9216, 9216),
             ("2Mx576_packed", np.arange(2 * n, dtype=np.uint64) * 576, np.full(2 * n, 556, np.uint32), 2 * n * 576,
              576)]   # small packets: the balanced kernel (k_ipv4_lb)
    # the flush mix of bench.py's wire_mix leg (control segments and data, packed 16-B aligned)
    import bench
    mix_segs, mix_region = bench.wire_mix_segments(n)
    works.append(("1M_flush_mix", mix_segs, None, mix_region, 1500))
    only = os.environ.get("WIRE_AB_ONLY")
    rounds = int(os.environ.get("WIRE_AB_ROUNDS", "5"))
    for name, offs, tl, rb, cap in works:
        if only and name not in only.split(","):
            continue
        if tl is None:   # ready TXSEG records
            segs = offs
            m = segs.size
            reg0 = torch.zeros(rb, dtype=torch.uint8, device=dev)
            tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), m, 1456, reg0, 0, None)
            offs = segs["out_off"].astype(np.uint64)
        else:
            reg0 = build(offs, tl, rb)
        m = offs.size
        doff = torch.from_numpy(offs.view(np.int64)).to(dev)
        regs = {k: reg0.clone() for k in libs}
        outs = {k: torch.empty(m, dtype=torch.int16, device=dev) for k in libs}
        stas = {k: torch.empty(m, dtype=torch.uint8, device=dev) for k in libs}

        def call(k, mode, reg=None):
            reg = regs[k] if reg is None else reg
            rc = libs[k].tcpcsum_ipv4_batch_dev(reg.data_ptr(), rb, doff.data_ptr(), m, cap, mode,
                                                outs[k].data_ptr(), stas[k].data_ptr(), h, None)
            assert rc == 0, (k, rc)

        same = {}
        for k in libs:
            call(k, 0)
        torch.cuda.synchronize()
        for k in libs:
            same[k] = bool(torch.equal(regs[k], regs["in_tree"]) and torch.equal(outs[k], outs["in_tree"]) and
                           torch.equal(stas[k], stas["in_tree"]))
        for k in libs:
            call(k, 1)
        torch.cuda.synchronize()
        for k in libs:
            same[k] = same[k] and bool((outs[k] == 0).all().item() and (stas[k] == 0).all().item())
        # every build is timed on one and the same region (filled: FILL rewrites the same bytes),
        # so that where a buffer lies in HBM is no difference between builds (a clone per build
        # made identical kernels differ by up to 5 %)
        regt = regs["in_tree"]
        res = {(k, md): [] for k in libs for md in (1, 0)}
        for _ in range(rounds):
            for k in libs:
                for md in (1, 0):
                    for _ in range(3):
                        call(k, md, regt)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(20):
                        call(k, md, regt)
                    e1.record(st)
                    torch.cuda.synchronize()
                    res[(k, md)].append(e0.elapsed_time(e1) / 20)
        for (k, md), ts in res.items():
            print(json.dumps({"measure": name, "build": k, "mode": "verify" if md else "fill",
                              "ms_median": round(statistics.median(ts), 4), "ms_min": round(min(ts), 4),
                              "same": same[k]}), flush=True)
        del regs, reg0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
