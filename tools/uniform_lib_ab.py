#!/usr/bin/env python3
"""Uniform kernel (tcpcsum_batch_uniform_dev) A/B: the in-tree library against other builds
(tools/ab_build.sh, e.g. measurement builds of TCPCSUM_LOAD_CPOL), interleaved in one process on
the same Appendix B batches (bench.py's headline and 64-B configs, rotating buffers; AB_LENS=a,b,...
adds ~1.5 GB batches of those segment lengths), HIP events on the launch stream. Every build's results must equal the in-tree build's. JSON lines.

  python tools/uniform_lib_ab.py tcp_amd/ab/libtcpcsum_X.so ...
"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import tcp_amd
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    libs = {"in_tree": tcp_amd.lib()}
    for p in sys.argv[1:]:
        lib = ctypes.CDLL(p)
        lib.tcpcsum_batch_uniform_dev.argtypes = [vp, u64, u32, vp, u32, vp, u64, vp, vp]
        lib.tcpcsum_batch_uniform_dev.restype = ctypes.c_int
        libs[os.path.basename(p).replace("libtcpcsum_", "").replace(".so", "")] = lib
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    cases = [("1Mx1500", 1 << 20, 1500, 2, 50), ("1Mx64", 1 << 20, 64, 32, 200)]
    for L in [int(x) for x in os.environ.get("AB_LENS", "").split(",") if x]:   # more sizes, ~1.5 GB each
        cases.append((f"len{L}", 1572864000 // L, L, 2, 30))
    for name, n, L, rot, steps in cases:
        bufs, sss = [], []
        for r in range(rot):
            d = torch.empty(n * L, dtype=torch.uint8, device=dev)
            tcp_amd.synth_fill(d, r * n * L, n * L)
            s = torch.empty(n, dtype=torch.int32, device=dev)
            tcp_amd.synth_pseudo(s, 0, n, L)
            bufs.append(d)
            sss.append(s)
        outs = {k: torch.empty(n, dtype=torch.int16, device=dev) for k in libs}

        def call(k, r):
            rc = libs[k].tcpcsum_batch_uniform_dev(bufs[r].data_ptr(), L, L, sss[r].data_ptr(), 0,
                                                   outs[k].data_ptr(), n, st.cuda_stream, None)
            assert rc == 0, (k, rc)
        for k in libs:
            call(k, 0)
        torch.cuda.synchronize()
        same = {k: bool(torch.equal(outs[k], outs["in_tree"])) for k in libs}
        times = {k: [] for k in libs}
        for _ in range(rounds):
            for k in libs:
                for i in range(5):
                    call(k, i % rot)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for i in range(steps):
                    call(k, i % rot)
                e1.record(st)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / steps)
        for k, ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"measure": name, "build": k, "ms_median": round(ms, 5), "ms_min": round(min(ts), 5),
                              "frac_of_8TBs": round(n * L / (ms * 1e-3) / 8e12, 4), "same": same[k]}), flush=True)
        del bufs, sss, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
