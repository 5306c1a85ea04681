#!/usr/bin/env python3
"""End-to-end (host-memory) rates of the checksum path: PCIe-inclusive.

The reference's packets start and end in host memory (raw-socket buffers).
This measures the library's host entry points on MI355X:
  * tcpcsum_batch_uniform_host over 1M x 1500 B in pageable memory (copied
    by the context's host threads into pinned staging, chunk k+1 while the
    kernel reads chunk k over PCIe) and in pinned memory (zero-copy: the
    kernel reads host memory over PCIe);
  * tcpcsum_ipv4_batch_host FILL on one releaseSend-sized batch (1024 packets
    of 1500 B, loop.c:27-94) in the reference's pool layout (32 KiB slots) and
    packed, pageable vs pinned — per-batch latency (--sweep: per wire kernel
    shape / window flag);
  * tcpcsum_ipv4_batch_ptrs_host FILL over 1024 separately allocated 32 KiB
    out-buffers (the loop's own layout, loop.c:180-183): malloc'd (packets
    copied into pinned staging, checks stored back) and carved from one
    tcpcsum_host_alloc pool (filled in place), for 1 / 2 / 4 / 8 copy threads
    (TCPCSUM_HOST_WIRE_THREADS) and spin vs blocking wait — wall time and the
    CPU time per batch (the calling thread + the copy threads, from the
    context's counters: "core-us");
  * the sendmmsg seam itself (tools/mmsg_bench under libtcpcsum_preload.so,
    the same variants, CPU time of the whole process per batch) beside the
    reference's CPU path for the same batch (one csum_continue per packet,
    -O2, one core).

  python tools/e2e.py  -> one JSON line per measurement
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def best_of(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), statistics.median(ts)


def main():
    import numpy as np
    import torch
    import tcp_amd
    from tests.packets import ip_packet

    rng = np.random.default_rng(1)
    n, L = 1 << 20, 1500
    nbytes = n * L
    ctx = tcp_amd.HostContext(0)
    pageable = np.empty(nbytes, np.uint8)
    pageable[:] = rng.integers(0, 256, nbytes, dtype=np.uint8)
    pinned = tcp_amd.pinned_empty(nbytes)
    pinned[:] = pageable
    ss = rng.integers(0, 393211, n, dtype=np.uint32)

    os.environ["TCPCSUM_HOST_PINNED_DMA"] = "0"
    ctx_inplace = tcp_amd.HostContext(0)   # page-locked batches read in place over PCIe (round 3's path)
    os.environ.pop("TCPCSUM_HOST_PINNED_DMA", None)
    for rnd in range(2):   # interleaved
        for name, buf, c in (("pageable", pageable, ctx), ("pinned_dma", pinned, ctx),
                             ("pinned_zero_copy", pinned, ctx_inplace)):
            c.batch_uniform(buf, L, L, n, ss)   # warm
            s0 = c.stats()
            tmin, tmed = best_of(lambda: c.batch_uniform(buf, L, L, n, ss), 5)
            s1 = c.stats()
            cpu = (s1["ns_cpu_caller"] - s0["ns_cpu_caller"] + s1["ns_cpu_workers"] - s0["ns_cpu_workers"]) / 5e9
            print(json.dumps({"measure": "uniform_host_1Mx1500", "memory": name, "round": rnd, "best_s": round(tmin, 5),
                              "GiB/s_best": round(nbytes / tmin / 2**30, 2),
                              "GiB/s_median": round(nbytes / tmed / 2**30, 2), "core_s_per_call": round(cpu, 4)}),
                  flush=True)
    ctx_inplace.close()

    # raw PCIe reference: one pinned H2D copy of the same bytes
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(pinned)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()

    def h2d():
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
    tmin, _ = best_of(h2d, 5)
    print(json.dumps({"measure": "raw_h2d_pinned_copy", "GiB/s_best": round(nbytes / tmin / 2**30, 2)}), flush=True)
    del dst

    # one releaseSend batch: 1024 packets, 1456-B payload -> 1500-B IP packets
    for layout, slot in (("pool_32KiB_slots", 32768), ("packed_1500B", 1500)):
        # full-size packets: 20 B IP + 24 B TCP + 1456 B payload = 1500 B each
        pkts = [np.frombuffer(ip_packet(rng, 1456), np.uint8) for _ in range(1024)]
        assert all(p.size == 1500 for p in pkts)
        reg = np.zeros(1024 * slot, np.uint8)
        offs = np.arange(1024, dtype=np.uint64) * np.uint64(slot)
        for i, p in enumerate(pkts):
            reg[i * slot:i * slot + p.size] = p
        pin = tcp_amd.pinned_empty(reg.size)
        pin[:] = reg
        variants = ([(sh, fl) for sh in (-1, 0, 1, 3, 5) for fl in (0, tcp_amd.TUNE_WIN16)]
                    if "--sweep" in sys.argv else [(-1, 0)])
        for name, r in (("pageable", reg), ("pinned_zero_copy", pin)):
            for sh, fl in variants:
                ctx.set_tuning(0, 0, sh, fl)
                ctx.ipv4_batch(r, offs, 32768, tcp_amd.IPV4_FILL)
                tmin, tmed = best_of(lambda: ctx.ipv4_batch(r, offs, 32768, tcp_amd.IPV4_FILL), 50)
                print(json.dumps({"measure": "ipv4_fill_host_1024x1500", "layout": layout, "memory": name,
                                  "shape": sh, "flags": fl,
                                  "us_best": round(tmin * 1e6, 1), "us_median": round(tmed * 1e6, 1),
                                  "region_bytes": int(r.size),
                                  "GiB/s_packet_bytes_median": round(1024 * 1500 / tmed / 2**30, 2)}),
                      flush=True)
            ctx.set_tuning(0, 0, -1, 0)

    # the loop's own layout: 1024 separate 32 KiB buffers, in and out alternating (malloc'd), or the
    # out-buffers carved from one page-locked pool (INTEGRATION.md level 2)
    bufs = []
    for i in range(2048):
        b = np.empty(32768, np.uint8)
        if i & 1:
            p = np.frombuffer(ip_packet(rng, 1456), np.uint8)
            b[:p.size] = p
        bufs.append(b)
    outb = bufs[1::2]
    pool = tcp_amd.pinned_empty(1024 * 32768)
    for k, b in enumerate(outb):
        pool[k * 32768:(k + 1) * 32768] = b
    lens = np.full(1024, 1500, np.uint32)
    ctx.close()
    reps = 200
    for layout, ptrs in (("malloc", np.array([b.ctypes.data for b in outb], np.uint64)),
                         ("pinned_pool", np.array([pool.ctypes.data + k * 32768 for k in range(1024)], np.uint64))):
        for threads, blocks in (((1, 1), (1, 2), (1, 4), (2, 1), (4, 1), (8, 1)) if layout == "malloc" else ((1, 1),)):
            for wait in ("spin", "block"):
                os.environ["TCPCSUM_HOST_WIRE_THREADS"] = str(threads)
                os.environ["TCPCSUM_HOST_STAGE_BLOCKS"] = str(blocks)
                ctx = tcp_amd.HostContext(0, blocking_wait=(wait == "block"))
                t0 = time.perf_counter()
                ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL)
                first = time.perf_counter() - t0
                s0 = ctx.stats()
                tmin, tmed = best_of(lambda: ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL), reps)
                s1 = ctx.stats()
                print(json.dumps({"measure": "ipv4_fill_ptrs_host_1024x1500", "layout": layout, "wait": wait,
                                  "copy_threads": s1["copy_threads"], "stage_blocks": blocks,
                                  "first_batch_us": round(first * 1e6, 1), "us_best": round(tmin * 1e6, 1),
                                  "us_median": round(tmed * 1e6, 1),
                                  "cpu_caller_us_per_batch": round((s1["ns_cpu_caller"] - s0["ns_cpu_caller"]) / reps / 1e3, 1),
                                  "cpu_workers_us_per_batch": round((s1["ns_cpu_workers"] - s0["ns_cpu_workers"]) / reps / 1e3, 1),
                                  "in_place": s1["pkts_in_place"] - s0["pkts_in_place"],
                                  "staged": s1["pkts_staged"] - s0["pkts_staged"]}), flush=True)
                ctx.close()
    os.environ.pop("TCPCSUM_HOST_WIRE_THREADS", None)
    os.environ.pop("TCPCSUM_HOST_STAGE_BLOCKS", None)

    # the seam itself: the interposer's per-batch latency vs the reference's CPU path
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, "tools", "mmsg_bench")
    pre = os.path.join(repo, "tcp_amd", "libtcpcsum_preload.so")
    import subprocess
    variants = [("cpu_reference_O2", "cpu", {}, []), ("preload_off", "gpu", {"TCPCSUM_PRELOAD_TX": "off"}, [])]
    for wait in ("block", "spin"):
        for threads, blocks in ((1, 1), (1, 2), (1, 4), (2, 1), (4, 1), (8, 1)):
            variants.append((f"preload_fill_staged_t{threads}_b{blocks}_{wait}", "gpu",
                             {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_WAIT": wait,
                              "TCPCSUM_HOST_WIRE_THREADS": str(threads), "TCPCSUM_HOST_STAGE_BLOCKS": str(blocks)}, []))
        variants.append((f"preload_fill_pinned_pool_{wait}", "gpu",
                         {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_WAIT": wait}, ["pinned"]))
    for label, mode, env_extra, extra_args in variants:
        env = {k: v for k, v in os.environ.items() if not k.startswith(("TCPCSUM_PRELOAD", "TCPCSUM_HOST"))}
        if mode == "gpu":
            env.update({"LD_PRELOAD": pre, "TCPCSUM_PRELOAD_ANY_SOCKET": "1"})
        env.update(env_extra)
        r = subprocess.run([exe, mode, "300"] + extra_args, env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "{}"
        d = json.loads(line)
        d.update({"measure": "sendmmsg_seam_1024x1500", "variant": label, "rc": r.returncode})
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
