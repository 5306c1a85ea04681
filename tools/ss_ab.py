#!/usr/bin/env python3
"""Start values read fresh vs warm: the in-tree library against other builds (tools/ab_build.sh,
e.g. TCPCSUM_SS_LOAD variants), interleaved in one process.

The 64-B config's first read of a batch costs ~2.2 us per 64 MiB launch, and all of it is the
u32 start-value array (tools/runlen_ab.py --parts: scalar start 12.2 us, start values read once
before 12.4, nothing read before 14.5). Per round and build: every rotation's start values are
rewritten (as a loop's next batch would be), then one pass over the rotations is timed queued
behind a sleep kernel (no host gaps) — "fresh" — and a second pass right after — "warm".
Results of every build must equal the in-tree build's. JSON lines.

  python tools/ss_ab.py tcp_amd/ab/libtcpcsum_X.so ...
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
    cases = [("1Mx64", 1 << 20, 64, 32), ("1Mx1500", 1 << 20, 1500, 2), ("1Mx256", 1 << 20, 256, 8),
             ("1Mx576", 1 << 20, 576, 4)]
    for name, n, L, rot in cases:
        bufs, sss = [], []
        for r in range(rot):
            d = torch.empty(n * L, dtype=torch.uint8, device=dev)
            tcp_amd.synth_fill(d, r * n * L, n * L)
            s = torch.empty(n, dtype=torch.int32, device=dev)
            bufs.append(d)
            sss.append(s)
        outs = {k: torch.empty(n, dtype=torch.int16, device=dev) for k in libs}

        def call(k, r):
            rc = libs[k].tcpcsum_batch_uniform_dev(bufs[r].data_ptr(), L, L, sss[r].data_ptr(), 0,
                                                   outs[k].data_ptr(), n, st.cuda_stream, None)
            assert rc == 0, (k, rc)

        def regen():
            for r in range(rot):
                tcp_amd.synth_pseudo(sss[r], r * n, n, L)

        regen()
        for k in libs:
            call(k, 0)
        torch.cuda.synchronize()
        same = {k: bool(torch.equal(outs[k], outs["in_tree"])) for k in libs}
        times = {k: {"fresh": [], "warm": []} for k in libs}
        for _ in range(rounds):
            for k in libs:
                regen()
                torch.cuda.synchronize()
                for which in ("fresh", "warm"):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda._sleep(int(2e7))
                    e0.record(st)
                    for r in range(rot):
                        call(k, r)
                    e1.record(st)
                    torch.cuda.synchronize()
                    times[k][which].append(e0.elapsed_time(e1) / rot)
        for k, tw in times.items():
            f, w = statistics.median(tw["fresh"]), statistics.median(tw["warm"])
            print(json.dumps({"measure": name, "build": k, "fresh_us": round(f * 1e3, 2), "warm_us": round(w * 1e3, 2),
                              "fresh_frac_of_8TBs": round(n * L / (f * 1e-3) / 8e12, 4),
                              "warm_frac_of_8TBs": round(n * L / (w * 1e-3) / 8e12, 4), "same": same[k]}), flush=True)
        del bufs, sss, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
