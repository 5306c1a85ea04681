#!/usr/bin/env python3
"""Segment builder (tcpcsum_tx_build_dev, k_tx_build) A/B: the in-tree library
against builds in tcp_amd/ab/, interleaved in one process on the same inputs
(1M x 1456-B payloads -> 1500-B packets, as tools/txbench.py), HIP events on
the launch stream. JSON lines: per build, median / min ms over the rounds, and
whether its packets and checks equal the in-tree build's (knock-out builds are
wrong by construction: `same` false).

  python tools/tx_ab.py --build [KO ...]   (CPU: compile tcp_amd/ab/libtcpcsum_txko<KO>.so,
                                             the kernels with -DTCPCSUM_TX_KNOCKOUT=<KO>)
  python tools/tx_ab.py [lib.so ...]        (GPU; default: every tcp_amd/ab/libtcpcsum_tx*.so)
"""
import ctypes
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
AB = os.path.join(REPO, "tcp_amd", "ab")


def build(kos):
    os.makedirs(AB, exist_ok=True)
    subprocess.run(["make", "-C", REPO, "tcp_amd/libtcpcsum.so"], check=True)
    flags = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wno-unused-parameter", "-Wno-unused-value",
             "-Wno-unused-result", "-I" + os.path.join(REPO, "include")]
    procs = []
    for ko in kos:
        obj = os.path.join(AB, f"kernels_txko{ko}.o")
        procs.append((ko, obj, subprocess.Popen(["/opt/rocm/bin/hipcc"] + flags + ["-DTCPCSUM_MEASUREMENT_BUILD=1", f"-DTCPCSUM_TX_KNOCKOUT={ko}", "-c",
                      os.path.join(REPO, "tcp_amd", "csrc", "tcpcsum_kernels.hip"), "-o", obj])))
    objs = [os.path.join(REPO, "build", "obj", o) for o in ("tcpcsum_api.o", "tcpcsum_host.o", "scalar_dropin.o")]
    for ko, obj, p in procs:
        assert p.wait() == 0, ko
        so = os.path.join(AB, f"libtcpcsum_txko{ko}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so, obj] + objs +
                       ["-lpthread"], check=True)
        print(so)


def main():
    if "--build" in sys.argv:
        build([int(x) for x in sys.argv[sys.argv.index("--build") + 1:]] or [1, 2, 4, 8])
        return
    import numpy as np
    import torch
    import tcp_amd

    paths = sys.argv[1:] or sorted(glob.glob(os.path.join(AB, "libtcpcsum_tx*.so")))
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    libs = {"in_tree": tcp_amd.lib()}
    for p in paths:
        lib = ctypes.CDLL(p)
        lib.tcpcsum_tx_build_dev.argtypes = [vp, vp, u64, u32, vp, ctypes.c_int, vp, vp, vp]
        lib.tcpcsum_tx_build_dev.restype = ctypes.c_int
        libs[os.path.basename(p).replace("libtcpcsum_", "").replace(".so", "")] = lib
    L = int(os.environ.get("TX_LEN", "1456"))
    n = 1 << 20 if L == 1456 else max(1 << 16, min(1 << 22, (3 << 29) // max(L + 44, 1)))
    dev = torch.device("cuda:0")
    payload = torch.empty(n * L, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(payload, 0, n * L)
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = np.arange(n, dtype=np.uint64) * L
    segs["out_off"] = np.arange(n, dtype=np.uint64) * (L + 44)
    segs["saddr_be"] = 0x0100007F
    segs["daddr_be"] = np.arange(n, dtype=np.uint32)
    segs["seq"] = np.arange(n, dtype=np.uint32) * L
    segs["sport"], segs["dport"] = 4000, 45001
    segs["len"] = L
    segs["flags"] = tcp_amd.api.TXF_ACK | tcp_amd.api.TXF_DATA
    dsegs = torch.from_numpy(segs.view(np.uint8)).to(dev)
    outs = {k: torch.zeros(n * (L + 44), dtype=torch.uint8, device=dev) for k in libs}
    chks = {k: torch.zeros(n, dtype=torch.int16, device=dev) for k in libs}
    st = torch.cuda.current_stream()
    h = st.cuda_stream

    def call(k):
        rc = libs[k].tcpcsum_tx_build_dev(payload.data_ptr(), dsegs.data_ptr(), n, L, outs[k].data_ptr(), 0,
                                          chks[k].data_ptr(), h, None)
        assert rc == 0, (k, rc)

    for k in libs:
        call(k)
    torch.cuda.synchronize()
    same = {k: bool(torch.equal(outs[k], outs["in_tree"]) and torch.equal(chks[k], chks["in_tree"])) for k in libs}
    times = {k: [] for k in libs}
    for _ in range(int(os.environ.get("TX_AB_ROUNDS", "5"))):
        for k in libs:
            for _ in range(3):
                call(k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                call(k)
            e1.record(st)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20)
    moved = n * L + n * (L + 44) + n * 48
    for k, ts in times.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(json.dumps({"build": k, "ms_median": round(med, 4), "ms_min": round(ts[0], 4),
                          "GB/s_read+write": round(moved / (med * 1e-3) / 1e9, 1), "same": same[k]}), flush=True)


if __name__ == "__main__":
    main()
