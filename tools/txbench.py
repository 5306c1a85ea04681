#!/usr/bin/env python3
"""Throughput of the fused segment builder (tcpcsum_tx_build_dev) on MI355X.

1M descriptors, 1456-byte payloads (1500-byte IPv4 packets, the reference's
MTU) packed back to back, device-resident. The kernel reads each payload once
and writes each packet once: algorithmic bytes = payload read + packet write
(+48 B descriptor read). Compared with the unfused alternative: a device copy
of the payloads into place (torch copy_) plus the checksum kernel over the
built segments.

  python tools/txbench.py -> JSON lines   (--sweep: launch shapes; TX_LEN=payload bytes)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import tcp_amd

    # TX_LEN: payload bytes (default the MTU's 1456); n keeps ~1.5 GB of payload (>= 64K packets)
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
    out = torch.empty(n * (L + 44), dtype=torch.uint8, device=dev)
    chk = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.cuda.current_stream()

    def timeit(fn, steps=50):
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

    if "--sweep" in sys.argv:
        shapes = [int(x) for x in os.environ.get("TX_SHAPES", "0,1,2,3,4").split(",")]
        blocks = [int(x) for x in os.environ.get("TX_BLOCKS", "1024,4096,8192,16384,32768").split(",")]
        unrolls = [int(x) for x in os.environ.get("TX_UNROLLS", "1,2").split(",")]
        # TX_ROUNDS interleaved rounds over every variant, median per variant (shape -1: the plan's)
        variants = [(sh, mb, un) for sh in shapes for mb in blocks for un in unrolls]
        ts = {v: [] for v in variants}
        for _ in range(int(os.environ.get("TX_ROUNDS", "1"))):
            for v in variants:
                tcp_amd.set_tuning(v[1], v[2], v[0], 0)
                ts[v].append(timeit(lambda: tcp_amd.tx_build(payload, dsegs, n, L, out, 0, chk), 20))
        tcp_amd.set_tuning(0, 0, -1, 0)
        for (sh, mb, un), tl in ts.items():
            tt = sorted(tl)[len(tl) // 2]
            print(json.dumps({"sweep": "tx_build", "len": L, "n": n, "shape": sh, "max_blocks": mb, "unroll": un,
                              "ms": round(tt * 1e3, 4), "rounds": len(tl),
                              "GB/s": round((n * L + n * (L + 44) + n * 48) / tt / 1e9, 1)}), flush=True)
    # store policy: default vs non-temporal payload stores, interleaved rounds
    moved = n * L + n * (L + 44) + n * 48
    pol = {0: [], 128: [], 1024: []}
    for _ in range(5):
        for fl in pol:
            tcp_amd.set_tuning(0, 0, -1, fl)
            pol[fl].append(timeit(lambda: tcp_amd.tx_build(payload, dsegs, n, L, out, 0, chk), 20))
    tcp_amd.set_tuning(0, 0, -1, 0)
    for fl, ts in pol.items():
        ts.sort()
        print(json.dumps({"measure": "tx_build_store_policy", "flags": fl, "stores": {0: "default", 128: "nt", 1024: "write-through"}[fl],
                          "ms_median": round(ts[2] * 1e3, 4), "ms_min": round(ts[0] * 1e3, 4),
                          "GB/s_read+write": round(moved / ts[2] / 1e9, 1)}), flush=True)
    t = timeit(lambda: tcp_amd.tx_build(payload, dsegs, n, L, out, 0, chk))
    print(json.dumps({"measure": "tx_build_1Mx1456B", "kernel_ms": round(t * 1e3, 4),
                      "Mpkt/s": round(n / t / 1e6, 1), "GB/s_read+write": round(moved / t / 1e9, 1),
                      "frac_of_8TB/s": round(moved / t / 8e12, 4)}), flush=True)
    # unfused: copy payloads into the packet slots + checksum the built TCP segments
    outv = out.view(n, L + 44)
    pv = payload.view(n, L)
    ss = torch.zeros(n, dtype=torch.int32, device=dev)

    def unfused():
        outv[:, 44:].copy_(pv)
        tcp_amd.batch_uniform(out, L + 44, L + 24, n, ss, out=chk, offset=20)
    t2 = timeit(unfused)
    print(json.dumps({"measure": "unfused_copy_plus_checksum", "ms": round(t2 * 1e3, 4),
                      "fused_speedup": round(t2 / t, 2)}), flush=True)
    # practical ceiling for a read+write stream on this device: a contiguous copy
    src_c = payload[: n * L]
    dst_c = torch.empty_like(src_c)
    t3 = timeit(lambda: dst_c.copy_(src_c))
    print(json.dumps({"measure": "contiguous_copy_same_bytes", "ms": round(t3 * 1e3, 4),
                      "GB/s_read+write": round(2 * n * L / t3 / 1e9, 1)}), flush=True)
    del dst_c
    # correctness spot check on the device result: every packet verifies to zero
    offs = torch.from_numpy((np.arange(4096, dtype=np.uint64) * (L + 44)).view(np.int64)).to(dev)
    tcp_amd.tx_build(payload, dsegs, n, L, out, 0, chk)
    vout = torch.empty(4096, dtype=torch.int16, device=dev)
    vst = torch.empty(4096, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch(out, offs, 4096, 65535, tcp_amd.IPV4_VERIFY, vout, vst)
    print(json.dumps({"measure": "verify_first_4096", "all_zero": bool((vout == 0).all().item()),
                      "all_ok": bool((vst == 0).all().item())}))


if __name__ == "__main__":
    main()
