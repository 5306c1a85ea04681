#!/usr/bin/env python3
"""Fused builder (tcpcsum_tx_build_dev) and ragged-batch (tcpcsum_batch_desc_dev) A/B: the in-tree
library against other builds (tools/ab_build.sh), interleaved in one process on the same inputs,
HIP events on the launch stream. Every build's output must equal the in-tree build's. JSON lines.

  python tools/misc_lib_ab.py tcp_amd/ab/libtcpcsum_X.so ...

Workloads: tx_build of 1M packed 1456-B payloads into 1500-B packets (txbench.py's); ragged
batches of ~1.5 GB — packed IMIX-like lengths 40..1500 (the balanced kernel) and MTU-size
1400..1500 (lane groups)."""
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
    vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    libs = {"in_tree": tcp_amd.lib()}
    for p in sys.argv[1:]:
        lib = ctypes.CDLL(p)
        lib.tcpcsum_tx_build_dev.argtypes = [vp, vp, u64, u32, vp, ci, vp, vp, vp]
        lib.tcpcsum_batch_desc_dev.argtypes = [vp, vp, u64, u32, vp, vp, vp]
        libs[os.path.basename(p).replace("libtcpcsum_", "").replace(".so", "")] = lib
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    h = st.cuda_stream
    rounds = int(os.environ.get("AB_ROUNDS", "5"))

    def run(name, calls, outs, steps, algo_bytes):
        for k in libs:
            calls[k]()
        torch.cuda.synchronize()
        same = {k: all(torch.equal(a, b) for a, b in zip(outs[k], outs["in_tree"])) for k in libs}
        times = {k: [] for k in libs}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(rounds):
            for k in libs:
                for _ in range(3):
                    calls[k]()
                e0.record(st)
                for _ in range(steps):
                    calls[k]()
                e1.record(st)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / steps)
        for k, ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"measure": name, "build": k, "ms_median": round(ms, 5), "ms_min": round(min(ts), 5),
                              "GB_per_s": round(algo_bytes / (ms * 1e-3) / 1e9, 1), "same": same[k]}), flush=True)

    # tx_build: 1M x 1456-B payloads -> 1500-B packets, packed
    only = os.environ.get("MISC_AB_ONLY", "")
    n, L = 1 << 20, 1456
    if only and "tx_build_1Mx1456" not in only.split(","):
        n = 0
    payload = torch.empty(max(n, 1) * L, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, n * L)
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = np.arange(n, dtype=np.uint64) * L
    segs["out_off"] = np.arange(n, dtype=np.uint64) * (L + 44)
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, L, 1 | 16
    dsegs = torch.from_numpy(segs.view(np.uint8)).to(dev)
    pk = {k: torch.empty(n * (L + 44), dtype=torch.uint8, device=dev) for k in libs}
    ck = {k: torch.empty(n, dtype=torch.int16, device=dev) for k in libs}
    calls = {k: (lambda k=k: libs[k].tcpcsum_tx_build_dev(payload.data_ptr(), dsegs.data_ptr(), n, L,
                                                           pk[k].data_ptr(), 0, ck[k].data_ptr(), h, None))
             for k in libs}
    if n:
        run("tx_build_1Mx1456", calls, {k: (pk[k], ck[k]) for k in libs}, 20, n * (2 * L + 44))
    del payload, dsegs, pk, ck
    torch.cuda.empty_cache()

    # ragged descriptor batches
    rng = np.random.default_rng(5)
    for name, lo, hi in (("desc_imix_40_1500", 40, 1500), ("desc_mtu_1400_1500", 1400, 1500),
                         ("desc_small_40_200", 40, 200), ("desc_imix_a16_40_1500", 40, 1500)):
        if only and name not in only.split(","):
            continue
        lens = rng.integers(lo, hi + 1, 1 << 22).astype(np.uint32)
        # a16: every segment starting 16-B aligned (packets in malloc'd / 16-B packed buffers)
        span = (lens.astype(np.uint64) + 15) // 16 * 16 if "_a16_" in name else lens.astype(np.uint64)
        total = np.cumsum(span)
        m = int(np.searchsorted(total, 1572864000))
        lens = lens[:m]
        offs = np.concatenate([[0], np.cumsum(span[:m])[:-1]]).astype(np.uint64)
        data = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device=dev)
        tcp_amd.synth_fill(data, 0, data.numel())
        d = np.zeros(m, tcp_amd.DESC_DTYPE)
        d["offset"], d["len"], d["sum_start"] = offs, lens, np.arange(m, dtype=np.uint32) * 7
        dd = torch.from_numpy(d.view(np.uint8)).to(dev)
        outs = {k: torch.empty(m, dtype=torch.int16, device=dev) for k in libs}
        calls = {k: (lambda k=k: libs[k].tcpcsum_batch_desc_dev(data.data_ptr(), dd.data_ptr(), m, hi,
                                                                 outs[k].data_ptr(), h, None)) for k in libs}
        run(name, calls, {k: (outs[k],) for k in libs}, 20, int(lens.sum()))
        del data, dd, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
