#!/usr/bin/env python3
"""bench.py — GiB/s checksummed (device-resident) on MI355X, bit-exact TCP checksum.

BASELINE.json metric, measured on its configs[1]: 1M x 1500-byte synthetic
segments per GPU (SURVEY.md Appendix B generator), inputs resident in HBM
before the timed region. One step = one launch of the batch checksum
(tcpcsum_batch_uniform_dev: /root/reference/context.c:104-145 for every segment
of the batch) over the GPU's whole shard.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1500|64|64k]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Multi-GPU: one process per GPU, each owns a contiguous shard of segments
(weak scaling: 1M segments per GPU; N=8 is BASELINE's 8M x 1500 config). No
collective touches the data path (north_star: independent segment batches, no
RCCL): torch.distributed over gloo (CPU) only brackets the timed region with
barriers and takes the max over ranks of its duration and the min of the
per-rank digest checks. `python bench.py --gpus N` without a launcher starts
the N rank processes itself (before any GPU call) and relays rank 0's line.

Rank 0 prints one JSON line. ``roofline.achieved`` = algorithmic bytes per
launch (segments x segment bytes) / the kernel's average duration, measured
with HIP events on the stream the kernels are launched on. ``cpu_baseline``
times the oracle's C restatement of the reference's scalar checksum on this
host (rank 0, N=1 only), the only use of oracle/ in this file.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import resource
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

METRIC = "GiB/s checksummed (device-resident), 1500B & 64KiB segment batches; bit-exact"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (segments per GPU, segment bytes, description)
    "1500": (1 << 20, 1500, "1M x 1500-byte synthetic segments per GPU, device-resident"),
    "64": (1 << 20, 64, "1M x 64-byte header-only segments per GPU, device-resident (L3-rotated)"),
    "64k": (1 << 18, 65536, "256K x 64KiB jumbo segments per GPU, device-resident"),
}


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [s0, s0+cnt) of `total` segments for `rank` of `world`."""
    s0 = total * rank // world
    s1 = total * (rank + 1) // world
    return s0, s1 - s0


def dist_env() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def max_over_ranks(x: float, dist, device) -> float:
    if dist is None:
        return x
    import torch
    if dist.get_backend() == "gloo":
        device = torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_region(step, steps: int, warmup: int, dist, sync, on_start=None, on_end=None, after_first=None) -> float:
    """W untimed steps, then EXACTLY `steps` steps between barrier+sync on both sides.
    on_start/on_end run right after/before the syncs (HIP event records); after_first right after
    the first timed step is enqueued. Returns this rank's wall seconds for the timed steps."""
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if on_start:
        on_start()
    for i in range(steps):
        step()
        if i == 0 and after_first:
            after_first()
    if on_end:
        on_end()
    sync()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    return t1 - t0


def load_traffic(config: str):
    """HBM bytes per launch from the committed PMC summary (profiles/traffic.json), if present."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        v = d.get(config, {}).get("hbm_bytes_per_launch")
        return float(v) if v is not None else None
    except Exception:
        return None


def host_cpu_info() -> dict:
    """Model, sockets, physical cores and hardware threads of this host; the cgroup CPU quota."""
    model, sockets, cores = "", set(), set()
    phys = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and not model:
                    model = v
                elif k == "physical id":
                    phys = v
                    sockets.add(v)
                elif k == "core id":
                    cores.add((phys, v))
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return {"host_cpu": model, "sockets": len(sockets) or None, "physical_cores": len(cores) or None,
            "hw_threads": os.cpu_count(), "threads_in_affinity": avail, "cgroup_cpu_quota": quota}


def usable_cpus(info: dict) -> int:
    """Threads this job can run at once: the affinity mask, capped by a cgroup CPU quota (the GPU
    pool grants 16 CPUs of quota while the mask shows all 256 hardware threads)."""
    n = max(1, info["threads_in_affinity"] or 1)
    q = info["cgroup_cpu_quota"]
    if q:
        n = min(n, max(1, math.ceil(q)))
    return n


def cpu_baseline(seconds: float) -> dict:
    """The reference's scalar checksum (C restatement of context.c:104-145, oracle/) on this host, as
    BASELINE.md plans it, for each single-GPU config's segment size: gcc -O2 and -O0 -g (the
    reference Makefile sets no CFLAGS, Makefile:3), on 1 thread and on every CPU this job may use
    (usable_cpus). Each figure is >= 5 passes over the same host-resident batch, timed from before
    the workers are released to after the last one finishes; best and median pass reported, and
    `value` is the median at -O2 on the usable CPUs for the 1500-B config — a rate this job can
    sustain, not a lucky pass. Bounded sample: the 1500-B and 64-KiB batches are 1.5 GB (the
    1500-B one is exactly the GPU's batch) — a quarter of that on one thread — and the 64-B one is the
    GPU's 64 MiB batch."""
    import oracle
    info = host_cpu_info()
    T = usable_cpus(info)
    # (segment bytes, opt, threads, share of `seconds`)
    plan = [(1500, "O2", T, 0.25), (1500, "O2", 1, 0.15), (1500, "O0", 1, 0.1), (1500, "O0", T, 0.1),
            (64, "O2", T, 0.1), (64, "O2", 1, 0.05), (64, "O0", 1, 0.05),
            (65536, "O2", T, 0.1), (65536, "O2", 1, 0.05), (65536, "O0", 1, 0.05)]
    figures = {}
    digests = {}
    for L, opt, th, share in plan:
        # one thread gets a quarter of the batch (384 MB: still far past the host's caches)
        nseg = (1 << 20) if L <= 1500 else (3 << 29) // L
        if th == 1 and L > 64:
            nseg //= 4
        c0 = cgroup_cpu_stat()
        r = oracle.cpu_bench(th, L, nseg, seconds * share, opt)
        c1 = cgroup_cpu_stat()
        key = f"{L}B_{opt}_{'1thread' if th == 1 else f'{th}threads'}"
        figures[key] = {"best": round(r["best"], 3), "median": round(r["median"], 3), "passes": r["passes"],
                        "sample": f"{nseg} x {L} B", **cgroup_delta(c0, c1)}
        digests.setdefault((L, nseg), set()).add(r["digest"])   # same batch -> same results at any -O / threads
    head = figures[f"1500B_O2_{'1thread' if T == 1 else f'{T}threads'}"]
    thr = head.get("throttled_ms")
    return {
        "value": head["median"], "unit": "GiB/s", "cores": T, "kind": "port",
        "sample": (f"1M x 1500-byte segments (Appendix B stream, 1.5 GB in host DRAM, first touched by the "
                   f"thread that reads it), gcc -O2, {T} threads = the CPUs this job may use; median of "
                   f"{head['passes']} passes (best {head['best']})"),
        "threads": T,
        # whether the job's cgroup throttled the figure (cpu.stat deltas around it)
        "quota_limited_threads": T, "throttled_ms": thr, "nr_throttled": head.get("nr_throttled"),
        "throttle_note": (None if thr is None else
                          f"throttled {thr} ms in {head.get('nr_throttled')} of {head.get('nr_periods')} quota periods "
                          "while this figure ran" if thr > 0 else
                          "not throttled while this figure ran: its median/best spread is not the CPU quota"),
        "figures": figures,
        "digests_agree": all(len(v) == 1 for v in digests.values()),
        **info,
    }


def digest_matches(res, config: str, world: int, rank: int, per_gpu: int):
    """Rank `rank`'s results of rotation 0 vs the reference's Appendix B digest (None: no digest)."""
    import numpy as np
    gold = json.load(open(os.path.join(REPO, "tests", "golden", "reference_vectors.json")))["digests"]
    key = {("1500", 1): "1Mx1500", ("64", 1): "1Mx64", ("64k", 1): "256Kx64KiB"}.get((config, world))
    if config == "1500" and world > 1 and per_gpu == 1 << 20:
        key = f"8Mx1500_shard{rank}" if rank < 8 else None
    if not key:
        return None
    g = gold[key]
    return bool(int(res.astype(np.uint64).sum()) == g["sum"]
                and f"{int(np.bitwise_xor.reduce(res)):04x}" == g["xor"]
                and [f"{v:04x}" for v in res[:4]] == g["first4"] and f"{res[-1]:04x}" == g["last"])


def run_config(config: str, steps: int, warmup: int, rank: int, world: int, dist, device, rotate: int = 0,
               streams: int = 1, multi: int = 0):
    """Generate this rank's shard of `config` in HBM, check rotation 0 against the reference's
    digest, then time `steps` launches (after `warmup`) between barriers. multi = K > 0: each step
    is ONE launch over K distinct batches (tcpcsum_batch_uniform_multi_dev).
    Returns (result dict, rank's buffers for the probe)."""
    import numpy as np
    import torch
    import tcp_amd

    per_gpu, L, desc = CONFIGS[config]
    total = per_gpu * world
    s0, cnt = shard_range(total, world, rank)
    batch_bytes = cnt * L
    # Small batches would be served from the 256 MiB Infinity Cache on repeat
    # launches; rotate distinct batches so consecutive reads of the same bytes
    # are >= 2 GiB apart (measured effect at 1.5 GB: < 1 %).
    rot = max(1, math.ceil((2 << 30) / batch_bytes))
    if rotate:
        rot = rotate
    if multi:
        rot = max(rot, multi)
    stream = torch.cuda.current_stream()
    bufs, sss = [], []
    for r in range(rot):
        data = torch.empty(batch_bytes, dtype=torch.uint8, device=device)
        ss = torch.empty(cnt, dtype=torch.int32, device=device)
        # rotation r holds the same segment indices with the stream bytes of a later block
        tcp_amd.synth_fill(data, (s0 + r * total) * L, batch_bytes)
        tcp_amd.synth_pseudo(ss, s0, cnt, L)
        bufs.append(data)
        sss.append(ss)
    out = torch.empty(cnt, dtype=torch.int16, device=device)
    torch.cuda.synchronize()

    # Sanity (not a parity test — tests/ does that): rotation 0 of each shard is
    # exactly the Appendix B batch whose digest the reference produced.
    tcp_amd.batch_uniform(bufs[0], L, L, cnt, sss[0], out=out)
    torch.cuda.synchronize()
    res = out.cpu().numpy().view(np.uint16)
    try:
        check = digest_matches(res, config, world, rank, per_gpu)
    except Exception:
        check = None

    if dist is not None:   # the check holds only if it holds on every rank
        flag = 1.0 if check else (0.0 if check is False else -1.0)
        fl = -max_over_ranks(-flag, dist, device)   # min over ranks
        check = None if fl < 0 else bool(fl == 1.0)

    k = [0]
    # streams == 2: consecutive launches (distinct batches, distinct result arrays) alternate
    # between two streams, so launch k+1's ramp overlaps launch k's drain — independent
    # batches pipelined, as a loop flushing batch after batch would run them
    sts = [stream] + [torch.cuda.Stream(device=device) for _ in range(streams - 1)]
    outs = [out] + [torch.empty(cnt, dtype=torch.int16, device=device) for _ in range(streams - 1)]

    if multi:   # K batches per launch, each its own rotation and result array
        mouts = [out] + [torch.empty(cnt, dtype=torch.int16, device=device) for _ in range(multi - 1)]
        marr = [tcp_amd.ubatches([(bufs[(g * multi + j) % rot], L, L, cnt, sss[(g * multi + j) % rot], mouts[j])
                                  for j in range(multi)]) for g in range(max(1, rot // multi))]

    def step():
        r = k[0] % rot
        j = k[0] % streams
        k[0] += 1
        if multi:
            tcp_amd.batch_uniform_multi(marr[(k[0] - 1) % len(marr)], stream=sts[0])
        else:
            tcp_amd.batch_uniform(bufs[r], L, L, cnt, sss[r], out=outs[j], stream=sts[j])

    # HIP events on the launch stream(s) bracket the kernels of the timed region. The kernel's
    # average duration is taken over launches 2..K (from an event right after the first launch):
    # the first timed launch starts on an idle GPU only once the host has enqueued it, a gap
    # that is no part of any kernel (the host enqueues a launch in ~5 us, the 64-B kernel runs
    # 12.4 us: launches 2..K run back to back; profiles/r06_runlen.jsonl "cpu_enqueue").
    # window_ms_per_launch keeps the whole window / K beside it.
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in sts]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in sts]
    evA = torch.cuda.Event(enable_timing=True)

    def rec(evs):
        for e, st in zip(evs, sts):
            e.record(st)
    # torch creates a HIP event on its first record: do that here, not inside the timed region
    rec(ev0)
    rec(ev1)
    evA.record(sts[0])
    torch.cuda.synchronize()
    # warm-up: at least one launch over every rotation, so no timed launch is the first read of
    # a batch just generated — that read costs the 64-B config ~2 us per launch, all of it in the
    # freshly written start values (profiles/r06_first_read_parts.jsonl, r06_ss_ab.jsonl)
    warm = max(warmup, rot if not multi else len(marr))
    wall = timed_region(step, steps, warm, dist, torch.cuda.synchronize,
                        on_start=lambda: rec(ev0), on_end=lambda: rec(ev1),
                        after_first=(lambda: evA.record(sts[0])) if streams == 1 and steps > 1 else None)
    window_ms = max(ev0[0].elapsed_time(e) for e in ev1) / steps
    kernel_ms = evA.elapsed_time(ev1[0]) / (steps - 1) if streams == 1 and steps > 1 else window_ms
    wall_max = max_over_ranks(wall, dist, device)
    kernel_ms_max = max_over_ranks(kernel_ms, dist, device)
    if multi:   # batch 0 of group 0 is rotation 0 = the Appendix B batch
        tcp_amd.batch_uniform_multi(marr[0], stream=sts[0])
        torch.cuda.synchronize()
        try:
            mcheck = digest_matches(mouts[0].cpu().numpy().view(np.uint16), config, world, rank, per_gpu)
        except Exception:
            mcheck = None
        check = check and mcheck
    r = {"config": config, "desc": desc, "L": L, "cnt": cnt, "rot": rot, "batch_bytes": batch_bytes,
         "check": check, "wall_max": wall_max, "kernel_ms": kernel_ms, "kernel_ms_max": kernel_ms_max,
         "window_ms": window_ms, "warmup_launches": warm, "streams": streams, "multi": multi}
    return r, bufs, rot


def time_probe(bufs, nbytes: int, steps: int, device) -> float:
    """Average ms of the read-only probe (k_probe: the kernels' access shape, every byte read once)
    over the same rotation of batches a config's kernel was timed on, HIP events on the stream —
    as the kernel is timed: warm-up launches over every rotation, the same K launches, the
    average over launches 2..K."""
    import torch
    import tcp_amd
    pout = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=device)
    nb = (nbytes // 16) * 16
    for i in range(max(3, len(bufs))):
        tcp_amd.stream_probe(bufs[i % len(bufs)], nb, pout, tune=(0, 0, -1, 0))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    pe1, peA = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(steps):
        tcp_amd.stream_probe(bufs[i % len(bufs)], nb, pout, tune=(0, 0, -1, 0))
        if i == 0:
            peA.record(stream)
    pe1.record(stream)
    torch.cuda.synchronize()
    return peA.elapsed_time(pe1) / max(steps - 1, 1)


def time_wire(reg, doff, n: int, cap: int, tcp_bytes: int, built, period: int, steps: int, warmup: int,
              device) -> dict:
    """FILL and VERIFY (tcpcsum_ipv4_batch_dev) of the n packets at reg + doff[i], interleaved over 5
    rounds (3 untimed + `steps` timed launches each) with the same box's ceilings for their traffic
    over the same region: the read-only probe (every line read, as VERIFY) and the write-back probe
    (every line read and one whole 128-B line in `period` written back through, bytes unchanged —
    the FILL's HBM traffic without its arithmetic; TCPCSUM_TUNE_PROBE_WRITE). Median per mode: the
    first window after the build runs slow on some boxes (0.29 vs 0.245 ms VERIFY,
    tools/wire_fresh.py), which one window per mode would report as the kernel's rate. FILL must
    reproduce `built` (the fused builder's checks) for every packet, VERIFY must give 0."""
    import torch
    import tcp_amd
    out = torch.empty(n, dtype=torch.int16, device=device)
    sta = torch.empty(n, dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream()
    region = reg.numel()
    pout = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=device)
    # probe shape: one 4 KiB tile per wave in XCD order, the fastest found (0.2783 ms against 0.2834
    # for the best grid-stride shape, 8192 workgroups; profiles/r05_probe_rw_sweep.jsonl,
    # r05_probe_rw_xcd.jsonl)
    probe_rw = tcp_amd.make_tuning(0, 0, period, tcp_amd.TUNE_PROBE_WRITE)
    nb = (region // 16) * 16
    modes = (("fill", tcp_amd.IPV4_FILL), ("verify", tcp_amd.IPV4_VERIFY), ("copy_probe", None),
             ("read_probe", None))

    def launch(name, mode):
        if name == "copy_probe":
            tcp_amd.stream_probe(reg, nb, pout, tune=probe_rw)
        elif name == "read_probe":
            tcp_amd.stream_probe(reg, nb, pout, tune=(0, 0, -1, 0))
        else:
            tcp_amd.ipv4_batch(reg, doff, n, cap, mode, out, sta)
    res = {"algorithmic_bytes_per_launch": tcp_bytes}
    times = {name: [] for name, _ in modes}
    fill_ok = verify_ok = True
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    e1.record(stream)
    torch.cuda.synchronize()
    for _ in range(warmup):
        tcp_amd.ipv4_batch(reg, doff, n, cap, tcp_amd.IPV4_FILL, out, sta)
    for _ in range(5):
        for name, mode in modes:
            for _ in range(3):
                launch(name, mode)
            e0.record(stream)
            for _ in range(steps):
                launch(name, mode)
            e1.record(stream)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / steps)
            if name == "fill":
                fill_ok = fill_ok and bool(torch.equal(out, built)) and bool((sta == tcp_amd.PKT_OK).all())
            elif name == "verify":
                verify_ok = verify_ok and bool((out == 0).all()) and bool((sta == tcp_amd.PKT_OK).all())
    for name, _ in modes:
        ms = statistics.median(times[name])
        if name.endswith("probe"):
            moved = nb + (nb // (128 * period) * 128 if name == "copy_probe" else 0)
            res[name] = {"avg_ms": round(ms, 5), "ms_rounds": [round(t, 4) for t in times[name]],
                         "bytes_moved_per_launch": moved, "GB/s": round(moved / (ms * 1e-3) / 1e9, 1)}
            continue
        gbs = tcp_bytes / (ms * 1e-3) / 1e9
        res[name] = {"kernel_avg_ms": round(ms, 5), "kernel_ms_rounds": [round(t, 4) for t in times[name]],
                     "achieved_GB/s": round(gbs, 1), "roofline_frac": round(gbs / HBM_PEAK_GBS, 4)}
    res["copy_probe"]["what"] = (f"k_probe<4,WR>, one 4 KiB tile per wave in XCD order: every line of the "
                                 f"{region / 1e9:.2f} GB region read, one 128-B line in {period} written back "
                                 "through (sc0 sc1), bytes unchanged")
    res["read_probe"]["what"] = "k_probe<4>, one 4 KiB tile per wave in XCD order: every line of the region read"
    res["fill_over_verify"] = round(res["fill"]["kernel_avg_ms"] / res["verify"]["kernel_avg_ms"], 3)
    res["fill_over_copy_probe"] = round(res["fill"]["kernel_avg_ms"] / res["copy_probe"]["avg_ms"], 3)
    res["verify_over_read_probe"] = round(res["verify"]["kernel_avg_ms"] / res["read_probe"]["avg_ms"], 3)
    # the write-back probe rewrote the lines it read: the packets are still the builder's
    tcp_amd.ipv4_batch(reg, doff, n, cap, tcp_amd.IPV4_VERIFY, out, sta)
    torch.cuda.synchronize()
    verify_ok = verify_ok and bool((out == 0).all()) and bool((sta == tcp_amd.PKT_OK).all())
    res["check"] = fill_ok and verify_ok
    return res


def build_wire(segs, region_bytes: int, max_len: int, device):
    """The packets of TXSEG_DTYPE records `segs`, built on the GPU by the fused builder
    (context.c:150-213 on the device) from an Appendix B payload stream into a zeroed region:
    (region, device offsets, the builder's own checks, summed TCP bytes)."""
    import numpy as np
    import torch
    import tcp_amd
    n = len(segs)
    payload = torch.empty(1 << 26, dtype=torch.uint8, device=device)
    tcp_amd.synth_fill(payload, 0, payload.numel())
    reg = torch.zeros(region_bytes, dtype=torch.uint8, device=device)
    built = torch.empty(n, dtype=torch.int16, device=device)
    dsegs = torch.from_numpy(segs.view(np.uint8)).to(device)
    tcp_amd.tx_build(payload, dsegs, n, max_len, reg, 0, built)
    del dsegs, payload
    doff = torch.from_numpy(segs["out_off"].astype(np.uint64).view(np.int64)).to(device)
    tcp_bytes = int((24 + segs["len"].astype(np.int64) * ((segs["flags"] & tcp_amd.api.TXF_DATA) != 0)).sum())
    return reg, doff, built, tcp_bytes


def run_wire(steps: int, warmup: int, device) -> dict:
    """The reference's own operation on wire packets, device-resident, beside the headline:
    1M IPv4/TCP packets of 1500 B (1480 TCP bytes) framed as context.c:169-206 frames them, one
    per 1536-B slot, checks filled in place (context.c:208-209, tcpcsum_ipv4_batch_dev FILL) and
    verified (VERIFY). Built on the GPU by the fused builder, whose own checks are the anchor:
    FILL must reproduce them for every packet and VERIFY must then give 0 (a self-consistency
    check across two kernels, not a parity test — tests/ does that against the oracle).
    Algorithmic bytes = the 1480 TCP bytes each packet's checksum reads."""
    import numpy as np
    import tcp_amd

    n, slot, tot = 1 << 20, 1536, 1500
    tcp_len = tot - 20
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = (np.arange(n, dtype=np.uint64) * 4096) % np.uint64((1 << 26) - 65536)
    segs["out_off"] = np.arange(n, dtype=np.uint64) * slot
    segs["saddr_be"] = 0x0100007F
    segs["daddr_be"] = np.arange(n, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tcp_len - 24, 1 | 16
    reg, doff, built, tcp_bytes = build_wire(segs, n * slot, tcp_len - 24, device)
    assert tcp_bytes == n * tcp_len
    res = {"workload": "1M x 1500-B IPv4/TCP packets (context.c:169-206 framing) in 1536-B slots, "
                       "device-resident, checks filled / verified in place (tcpcsum_ipv4_batch_dev)"}
    res.update(time_wire(reg, doff, n, slot, tcp_bytes, built, slot // 128, steps, warmup, device))
    # HBM bytes actually moved (committed PMC pass: whole 128-B lines read, FILL's check lines
    # written back whole) per launch time — the FILL is a read+write stream, whose measured
    # ceiling is a plain copy's ~6.1 TB/s (tools/copy_probe.hip), not the 8 TB/s read peak
    try:
        with open(os.path.join(REPO, "profiles", "traffic.json")) as f:
            t = json.load(f)["wire_fill_1Mx1500"]
        rd, wr = t["read_bytes_per_launch"], t["write_bytes_per_launch_line_store"]
        res["fill"]["hbm_traffic_GB/s"] = round((rd + wr) / (res["fill"]["kernel_avg_ms"] * 1e-3) / 1e9, 1)
        res["verify"]["hbm_traffic_GB/s"] = round(
            (rd + t["write_bytes_per_launch_verify"]) / (res["verify"]["kernel_avg_ms"] * 1e-3) / 1e9, 1)
        res["traffic_source"] = "profiles/traffic.json wire_fill_1Mx1500 (rocprofv3 --pmc, round 5)"
    except Exception:
        pass
    return res


def wire_mix_segments(n: int):
    """The flush releaseSend (loop.c:27-94) hands sendmmsg on an echo server, as TXSEG_DTYPE records:
    of every 8 packets, 3 pure ACKs (context.c:558), one SYN-ACK (context.c:324, resent at :94) or
    FIN-ACK (:368) in turn — 44-B packets, a 24-B TCP header with the window-scale option — and 4
    data segments (socket.c:17) with 0..1456-B payloads (1500-B MTU), hash-spread. Packed back to
    back, each packet starting 16-B aligned as a malloc'd out-buffer does (loop.c:180-183)."""
    import numpy as np
    import tcp_amd
    i = np.arange(n, dtype=np.uint64)
    h = ((i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)
    kind = (i % np.uint64(8)).astype(np.int64)
    data = kind >= 4
    plen = np.where(data, (h % np.uint64(1457)).astype(np.int64), 0)
    flags = np.where(data, tcp_amd.api.TXF_DATA | tcp_amd.api.TXF_ACK,
                     np.where(kind == 3, np.where((i // np.uint64(8)) % np.uint64(2) == 0,
                                                  tcp_amd.api.TXF_SYN | tcp_amd.api.TXF_ACK,
                                                  tcp_amd.api.TXF_FIN | tcp_amd.api.TXF_ACK), tcp_amd.api.TXF_ACK))
    size = 44 + plen
    span = (size + 15) // 16 * 16
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    segs["out_off"] = np.concatenate([[0], np.cumsum(span)[:-1]]).astype(np.uint64)
    segs["payload_off"] = (i * np.uint64(4096)) % np.uint64((1 << 26) - 65536)
    segs["saddr_be"] = 0x0100007F
    segs["daddr_be"] = i.astype(np.uint32)
    segs["seq"] = (h & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    segs["ack"] = (i * np.uint64(7919)).astype(np.uint32)
    segs["sport"], segs["dport"] = 4000, 45001
    segs["len"], segs["flags"] = plen, flags
    return segs, int(span.sum())


def run_wire_mix(steps: int, warmup: int, device) -> dict:
    """the reference's real flush, not uniform MTU packets — 1M IPv4/TCP packets of
    the wire_mix_segments mix, device-resident, FILL and VERIFY in place (tcpcsum_ipv4_batch_dev:
    the balanced kernel k_ipv4_lb takes large batches of small or mixed packets), with the read
    and write-back probes over the same region. Algorithmic bytes = each packet's TCP bytes."""
    n = 1 << 20
    segs, region = wire_mix_segments(n)
    reg, doff, built, tcp_bytes = build_wire(segs, region, 1456, device)
    import tcp_amd
    ctl = int(((segs["flags"] & tcp_amd.api.TXF_DATA) == 0).sum())
    res = {"workload": (f"1M IPv4/TCP packets as releaseSend flushes them: {ctl} 44-B control segments (pure ACK, "
                        f"SYN-ACK, FIN-ACK) and {n - ctl} data segments of 0-1456-B payload, packed 16-B aligned "
                        f"({region / 1e6:.1f} MB, mean {region / n:.0f} B per packet), checks filled / verified "
                        "in place (tcpcsum_ipv4_batch_dev)")}
    res.update(time_wire(reg, doff, n, 1500, tcp_bytes, built, max(1, round(region / n / 128)), steps, warmup,
                         device))
    return res


def gpu_numa_cpus(device_index: int):
    """(NUMA node, CPUs of that node this process may use) of GPU `device_index`, from sysfs via its
    PCI address; (None, None) when unknown."""
    import torch
    try:
        p = torch.cuda.get_device_properties(device_index)
        bus = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        node = int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
        if node < 0:
            return None, None
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        return node, (cpus or None)
    except Exception:
        return None, None


def gather_walls(wall: float, dist, world: int) -> list:
    """Every rank's wall time, on every rank (gloo object gather; [wall] without a group)."""
    if dist is None:
        return [wall]
    walls = [None] * world
    dist.all_gather_object(walls, wall)
    return walls


def page_node_of(arr) -> int | None:
    """NUMA node of the first page of a numpy array (get_mempolicy MPOL_F_NODE|MPOL_F_ADDR), or None."""
    import ctypes
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        node = ctypes.c_int(-1)
        # SYS_get_mempolicy = 239 on x86-64; flags MPOL_F_NODE | MPOL_F_ADDR = 3
        if libc.syscall(239, ctypes.byref(node), None, ctypes.c_ulong(0), ctypes.c_void_p(arr.ctypes.data),
                        ctypes.c_ulong(3)) != 0:
            return None
        return node.value
    except Exception:
        return None


def page_node_shares(arr, samples: int = 512) -> dict | None:
    """Where a numpy array's pages live: share of `samples` pages spread over it per NUMA node
    (move_pages with no target nodes reports each page's node), or None."""
    import ctypes
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        base, nbytes = arr.ctypes.data, arr.nbytes
        npg = max(1, nbytes // 4096)
        idx = sorted({i * npg // samples for i in range(min(samples, npg))})
        pages = (ctypes.c_void_p * len(idx))(*[base + i * 4096 for i in idx])
        status = (ctypes.c_int * len(idx))()
        # SYS_move_pages = 279 on x86-64; nodes = NULL: query only
        if libc.syscall(279, 0, ctypes.c_ulong(len(idx)), pages, None, status, 0) != 0:
            return None
        out = {}
        for st in status:
            k = str(st) if st >= 0 else "err"
            out[k] = out.get(k, 0) + 1
        return {k: round(v / len(idx), 3) for k, v in sorted(out.items())}
    except Exception:
        return None


def node_free_gib() -> dict | None:
    """MemFree per NUMA node (sysfs), GiB, or None."""
    try:
        import glob
        out = {}
        for f in sorted(glob.glob("/sys/devices/system/node/node*/meminfo")):
            node = f.split("/")[-2][4:]
            for line in open(f):
                if "MemFree:" in line:
                    out[node] = round(int(line.split()[-2]) / (1 << 20), 1)
        return out or None
    except Exception:
        return None


def cgroup_cpu_stat() -> dict | None:
    """The job's cgroup cpu.stat counters (nr_periods, nr_throttled, throttled_usec, usage_usec), or None."""
    try:
        out = {}
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            out[k] = int(v)
        return out
    except Exception:
        return None


def cgroup_delta(c0, c1) -> dict:
    """Throttling between two cgroup_cpu_stat() reads: throttled ms, throttled periods, periods."""
    if not c0 or not c1:
        return {}
    d = {k: c1.get(k, 0) - c0.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")}
    return {"throttled_ms": round(d["throttled_usec"] / 1e3, 1), "nr_throttled": d["nr_throttled"],
            "nr_periods": d["nr_periods"], "cpu_usage_s": round(d["usage_usec"] / 1e6, 2)}


def cgroup_throttled_us() -> int | None:
    """The job's cgroup CPU throttling so far (cpu.stat throttled_usec), or None."""
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k == "throttled_usec":
                return int(v)
    except Exception:
        pass
    return None


def thp_share(arr) -> float | None:
    """Share of the array's mapping backed by transparent huge pages (/proc/self/smaps AnonHugePages
    over Rss of the VMA holding its first byte), or None."""
    a = arr.ctypes.data
    try:
        cur = None
        with open("/proc/self/smaps") as f:
            for line in f:
                head = line.split()
                if "-" in head[0] and len(head) >= 5 and all(c in "0123456789abcdef-" for c in head[0]):
                    lo, hi = (int(x, 16) for x in head[0].split("-"))
                    cur = {} if lo <= a < hi else None
                elif cur is not None and head[0] in ("Rss:", "AnonHugePages:"):
                    cur[head[0]] = int(head[1])
                    if len(cur) == 2:
                        return round(cur["AnonHugePages:"] / max(cur["Rss:"], 1), 3)
    except Exception:
        pass
    return None


def host_path_rate(bytes_per_rank: list, walls: list, steps: int) -> dict:
    """Whole-job end-to-end rate: every rank's bytes x steps over the slowest rank's wall time."""
    wmax = max(walls)
    return {"GiB/s": round(sum(bytes_per_rank) * steps / wmax / (1 << 30), 2),
            "per_rank_GiB/s": [round(b * steps / w / (1 << 30), 2) for b, w in zip(bytes_per_rank, walls)],
            "wall_max_s": round(wmax, 6)}


def host_context(local: int):
    """The host leg's context: blocking (sleeping) wait; its staging and HBM slots allocated by one
    warm batch past two full staging chunks (2 x 128 MiB) over a pinned buffer and a pageable one,
    so that, created at the start of the run as an application creates it at start-up, nothing it
    holds is allocated after the device legs have churned the allocators."""
    import numpy as np
    import tcp_amd
    ctx = tcp_amd.HostContext(local, blocking_wait=True)   # sleep, not spin, while the GPU works
    # the pageable ramp is 16, 32, 64 then 128 MiB chunks: past 2 full chunks both staging slots
    # reach their full size; pinned batches past 2 x 16 MiB take the DMA path (256 MiB pieces)
    warm = (16 + 32 + 64 + 128 + 128) << 20
    pin = tcp_amd.pinned_empty(warm)
    pin[:] = 0
    ctx.batch_uniform(pin, 1500, 1500, warm // 1500, 0)
    ctx.batch_uniform(np.zeros(warm, np.uint8), 1500, 1500, warm // 1500, 0)
    return ctx


def run_host_path(steps: int, warmup: int, rank: int, world: int, local: int, dist, device,
                  memory: str = "pageable", ctx=None) -> dict:
    """The path as north_star states it — starting and ending in host memory (raw-socket buffers) —
    one context per GPU (tcpcsum_ctx_*), every rank at once. Rank r owns its contiguous shard of
    the global 1500-B config (N=8: BASELINE's 8M x 1500 config, Appendix B shard r), held in host
    memory first touched from the CPUs of its GPU's NUMA node (the calling thread is moved there;
    the context pins its copy threads there and its pinned staging comes from hipHostMalloc for
    the current device). memory="pageable": each step is tcpcsum_batch_uniform_host over the
    pageable shard (copied by the context's threads into pinned staging chunk by chunk, DMA to
    HBM, kernel, results back into host memory); "pinned": the shard lives in tcpcsum_host_alloc
    memory and goes to HBM by DMA straight from those pages. The context sleeps while the GPU works
    (TCPCSUM_CTX_BLOCKING_WAIT), so cpu_core_s_per_step is the copying and launching only.
    Inputs and results in host memory: PCIe and
    host DRAM are the bound, not HBM. Rank 0 returns the whole-job rate, every
    rank's results checked against its Appendix B digest."""
    import numpy as np
    import torch
    import tcp_amd

    per_gpu, L, _ = CONFIGS["1500"]
    total = per_gpu * world
    s0, cnt = shard_range(total, world, rank)
    nbytes = cnt * L
    node, cpus = gpu_numa_cpus(local)
    saved = os.sched_getaffinity(0)
    if cpus and os.environ.get("TCPCSUM_BENCH_HOST_NUMA", "1") != "0":
        os.sched_setaffinity(0, cpus)
    try:
        # generated in HBM (Appendix B stream), then copied into host memory first touched here
        d = torch.empty(nbytes, dtype=torch.uint8, device=device)
        tcp_amd.synth_fill(d, s0 * L, nbytes)
        dss = torch.empty(cnt, dtype=torch.int32, device=device)
        tcp_amd.synth_pseudo(dss, s0, cnt, L)
        free_before = node_free_gib()
        host = tcp_amd.pinned_empty(nbytes) if memory == "pinned" else np.empty(nbytes, np.uint8)
        host[::4096] = 0   # first touch, page by page, from this node
        torch.from_numpy(host).copy_(d)
        ss = dss.cpu().numpy().view(np.uint32).copy()
        del d, dss
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        own_ctx = ctx is None
        if own_ctx:
            ctx = tcp_amd.HostContext(local, blocking_wait=True)   # sleep, not spin, while the GPU works
        try:
            res = ctx.batch_uniform(host, L, L, cnt, ss)
            try:
                check = digest_matches(res, "1500", world, rank, per_gpu)
            except Exception:
                check = None
            if dist is not None:
                flag = 1.0 if check else (0.0 if check is False else -1.0)
                fl = -max_over_ranks(-flag, dist, device)
                check = None if fl < 0 else bool(fl == 1.0)
            s_before = ctx.stats()
            ru0, thr0 = resource.getrusage(resource.RUSAGE_SELF), cgroup_throttled_us()
            wall = timed_region(lambda: ctx.batch_uniform(host, L, L, cnt, ss), steps, warmup, dist, lambda: None)
            ru1, thr1 = resource.getrusage(resource.RUSAGE_SELF), cgroup_throttled_us()
            s_after = ctx.stats()
            proc_cpu = (ru1.ru_utime + ru1.ru_stime) - (ru0.ru_utime + ru0.ru_stime)
            data_node = page_node_of(host)
            data_nodes = page_node_shares(host)
            thp = thp_share(host) if memory == "pageable" else None
        finally:
            if own_ctx:
                ctx.close()
        # the link's own rate, same rank, same moment: a raw DMA of the pinned shard to HBM
        # (every rank at once, between barriers), the ceiling both legs are held against
        raw = None
        if memory == "pinned":
            dst = torch.empty(nbytes, dtype=torch.uint8, device=device)
            src = torch.from_numpy(host)
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            rwall = timed_region(lambda: dst.copy_(src, non_blocking=True), 3, 1, dist, torch.cuda.synchronize)
            raw = host_path_rate([nbytes] * world, gather_walls(rwall, dist, world), 3)["GiB/s"]
            del dst
            torch.cuda.empty_cache()
    finally:
        os.sched_setaffinity(0, saved)
    walls = gather_walls(wall, dist, world)
    # every rank's cgroup CPU throttling over its timed region (a rank's cgroup may be the job's:
    # then they all report the same counter's growth)
    thr = None if thr0 is None or thr1 is None else round((thr1 - thr0) / 1e3, 1)
    throttled = gather_walls(thr, dist, world)
    calls = max(steps + warmup, 1)   # the stats and rusage deltas span the warm-up calls too
    cpu_ns = (s_after["ns_cpu_caller"] - s_before["ns_cpu_caller"]) + (s_after["ns_cpu_workers"] - s_before["ns_cpu_workers"])
    r = {"workload": f"{cnt} x {L}-byte segments per GPU in {memory} host memory "
                     f"({'Appendix B shard ' + str(rank) + ' of ' + str(total) if world > 1 else 'Appendix B 1M x 1500'}), "
                     "results back in host memory (tcpcsum_batch_uniform_host)",
         "memory": memory, "steps": steps, **host_path_rate([nbytes] * world, walls, steps),
         "digest_check": check, "numa_node_rank0": node, "copy_threads": s_after["bulk_threads"],
         "staging_numa_node_rank0": s_after["staging_numa_node"], "data_numa_node_rank0": data_node,
         "raw_pinned_h2d_GiB/s": raw, "data_thp_share": thp, "data_page_node_shares_rank0": data_nodes,
         "node_free_gib_before_rank0": free_before,
         "process_cpu_core_s_per_step_rank0": round(proc_cpu / calls, 4),
         "copy_ms_per_step_rank0": round((s_after["ns_copy"] - s_before["ns_copy"]) / calls / 1e6, 3),
         "wait_ms_per_step_rank0": round((s_after["ns_wait"] - s_before["ns_wait"]) / calls / 1e6, 3),
         "cgroup_throttled_ms_per_rank": throttled,
         "copy_threads_per_rank": gather_walls(s_after["bulk_threads"], dist, world),
         "local_world_size": int(os.environ.get("LOCAL_WORLD_SIZE", "1")),
         "cpu_core_s_per_step_rank0": round(cpu_ns / calls / 1e9, 4)}
    if raw:
        r["frac_of_raw_pinned_h2d"] = round(r["GiB/s"] / raw, 3)
    return r


SEAM_VARIANTS = (
    # name, mmsg_bench args, interposer env (None: no interposer), what
    ("tx_reference_cpu", ["cpu"], None,
     "the reference: csum_continue(getPseudoHeaderSum(...)) per packet on one core (context.c:208, -O2)"),
    ("tx_staged", ["gpu"], {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_POOL": "0"},
     "sendmmsg seam, loop.c unedited: the loop's malloc'd out-buffers copied into pinned staging, GPU FILL, "
     "checks stored back"),
    ("tx_pool", ["gpu"], {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_POOL": "mmsg_bench"},
     "sendmmsg seam, loop.c unedited, TCPCSUM_PRELOAD_POOL: the loop's mallocs served from the interposer's "
     "page-locked arena, GPU FILL in place"),
    ("rx_plain", ["rx"], None, "recvmmsg of the 1024 datagrams alone"),
    ("rx_drop_staged", ["rx"], {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "drop",
                                "TCPCSUM_PRELOAD_POOL": "0"},
     "recvmmsg seam, rx drop: GPU VERIFY of every segment (staged), failing ones removed"),
    ("rx_drop_pool", ["rx"], {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "drop",
                              "TCPCSUM_PRELOAD_POOL": "mmsg_bench"},
     "the same, in place in the arena's in-buffers"),
    ("rx_cpu_verify", ["rxcpu"], None, "recvmmsg, then the reference's arithmetic verifying every segment on one core"),
)


def run_seam(iters: int = 300) -> dict:
    """the seam in the record — tools/mmsg_bench over UDP loopback (no root), 1024 x
    1500-B packets per batch in the reference's buffer layout (loop.c:180-183), every variant a child
    process of its own (started before this process makes any GPU call), the interposer preloaded
    on the child alone. Medians of `iters` batches: wall us and core-us (the whole child's CPU time:
    caller, copy threads, HIP's threads) per sendmmsg / recvmmsg of 1024 packets (loop.c:75 / :24)."""
    import re
    import subprocess
    exe = os.path.join(REPO, "tools", "mmsg_bench")
    pre = os.path.join(REPO, "tcp_amd", "libtcpcsum_preload.so")
    if not (os.path.exists(exe) and os.path.exists(pre)):
        return {"error": "tools/mmsg_bench or tcp_amd/libtcpcsum_preload.so not built (make)"}
    base_env = {k: v for k, v in os.environ.items() if not k.startswith("TCPCSUM_PRELOAD") and k != "LD_PRELOAD"}
    out = {"batch": "1024 x 1500-B IPv4/TCP packets, one per 32 KiB malloc'd buffer (loop.c:180-183), UDP loopback",
           "iters": iters}
    for name, args, env_extra, what in SEAM_VARIANTS:
        env = dict(base_env)
        if env_extra is not None:
            env.update({"LD_PRELOAD": pre, "TCPCSUM_PRELOAD_ANY_SOCKET": "1", "TCPCSUM_PRELOAD_STATS": "1",
                        **env_extra})
        try:
            r = subprocess.run([exe] + args + [str(iters)], env=env, capture_output=True, text=True, timeout=120)
            d = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {}
        except Exception as e:   # a failed variant is reported, never fatal to the bench
            out[name] = {"error": repr(e)[:200]}
            continue
        if r.returncode != 0:
            out[name] = {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-300:]}
            continue
        v = {"what": what, "median_us": d.get("median_us"), "min_us": d.get("min_us"),
             "core_us_median": d.get("cpu_us_median"), "first_us": d.get("first_us")}
        if d.get("call_errors"):
            out[name] = {"error": f"{d['call_errors']} of {iters} calls failed (no GPU path: ENXIO)",
                         "stderr_tail": r.stderr[-300:]}
            continue
        if "checks_match_cpu" in d:
            v["checks_match_cpu"] = d["checks_match_cpu"]
        if "batches_not_all_verified" in d:
            v["batches_not_all_verified"] = d["batches_not_all_verified"]
            v["short_batches"] = d.get("short_batches")
        m = re.search(r"in_place=(\d+) staged=(\d+)", r.stderr)
        if m:
            v["packets_in_place"], v["packets_staged"] = int(m.group(1)), int(m.group(2))
        m = re.search(r"pool on=(\d) served=(\d+)", r.stderr)
        if m and env_extra and env_extra.get("TCPCSUM_PRELOAD_POOL", "0") != "0":
            v["pool_on"], v["pool_served"] = int(m.group(1)), int(m.group(2))
        out[name] = v
    ref = (out.get("tx_reference_cpu") or {}).get("median_us")
    for k in ("tx_staged", "tx_pool"):
        if ref and (out.get(k) or {}).get("median_us"):
            out[k]["speedup_vs_reference_cpu"] = round(ref / out[k]["median_us"], 2)
    return out


def spawn_ranks(args, argv, script=None) -> int:
    """`bench.py --gpus N` with no launcher: start ranks 0..N-1 as child processes (this process
    has made no GPU call), rendezvous on 127.0.0.1, relay rank 0's JSON line, return the worst
    exit code. If a rank fails the others are stopped (by PID) instead of waiting in a barrier, and
    every failed rank's exit code and the tail of its stderr are written to this process's stderr
    (rank 0's stderr is relayed in any case)."""
    import socket
    import subprocess
    import tempfile
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, script or os.path.abspath(__file__)] + list(argv if argv is not None else sys.argv[1:])
    procs, errs = [], []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        err = tempfile.TemporaryFile()
        errs.append(err)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      stderr=err))
    rc = 0
    first_failed = None
    out0 = b""
    try:
        while True:
            codes = [p.poll() for p in procs]
            failed = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if failed:   # a rank died: the others would wait in a barrier for ever
                first_failed, rc = failed[0]
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.05)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        out0 = procs[0].stdout.read() if procs[0].stdout else b""
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for r, (p, err) in enumerate(zip(procs, errs)):
            err.seek(0)
            text = err.read().decode(errors="replace")
            err.close()
            if r == 0 and text:
                sys.stderr.write(text)
            if p.returncode not in (0, None) and (r != 0 or not text):
                tail = "\n".join(text.splitlines()[-30:])
                cause = " (first to fail)" if r == first_failed else " (stopped after another rank failed)" \
                    if first_failed is not None else ""
                sys.stderr.write(f"bench.py: rank {r} exited with code {p.returncode}{cause}; stderr tail:\n"
                                 f"{tail}\n")
            elif r == 0 and p.returncode not in (0, None):
                sys.stderr.write(f"bench.py: rank 0 exited with code {p.returncode}\n")
        sys.stderr.flush()
    sys.stdout.write(out0.decode())
    sys.stdout.flush()
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="1500")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the other BASELINE configs (64 B, 64 KiB) reported beside the headline at N=1")
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)   # the default now; old scripts pass it
    ap.add_argument("--no-probe", action="store_true",
                    help="skip the read-only stream probe timed beside the headline at N=1 (the same box's "
                         "practical read ceiling in the kernel's access shape)")
    ap.add_argument("--max-blocks", type=int, default=0)
    ap.add_argument("--unroll", type=int, default=0)
    ap.add_argument("--shape", type=int, default=-1)
    ap.add_argument("--flags", type=int, default=0, help="TCPCSUM_TUNE_* bits")
    ap.add_argument("--rotate", type=int, default=0, help="distinct batches to rotate (0 = auto)")
    ap.add_argument("--streams", type=int, default=1, choices=[1, 2],
                    help="2: consecutive launches alternate between two streams (pipelined batches)")
    ap.add_argument("--other", default="", help=argparse.SUPPRESS)   # A/B: comma list of other configs (+ "wire")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the end-to-end host-memory leg (pageable and pinned shards, every rank)")
    ap.add_argument("--host-path-only", action="store_true",
                    help="only the end-to-end host-memory leg: one JSON line for it (tools/e2e_multi.sh)")
    ap.add_argument("--host-steps", type=int, default=5)
    ap.add_argument("--host-ctx-early", action="store_true",
                    help="create (and warm) the host leg's context at the start of the run")
    ap.add_argument("--host-path-first", action="store_true",
                    help="run the host-memory leg before the device configs (A/B: DESIGN.md §7, 'Order')")
    ap.add_argument("--host-path-last", action="store_true", help=argparse.SUPPRESS)   # the default
    ap.add_argument("--no-seam", action="store_true",
                    help="skip the sendmmsg / recvmmsg seam leg (tools/mmsg_bench children, N=1)")
    ap.add_argument("--seam-iters", type=int, default=300)
    args = ap.parse_args(argv)

    rank, world, local = dist_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args, argv)   # before any GPU call in this process
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    # the seam's children run before this process makes any GPU call (N=1 only)
    seam = run_seam(args.seam_iters) if world == 1 and not args.no_seam and not args.host_path_only else None

    import numpy as np
    import torch
    import tcp_amd

    # Rehearsal knob for a 1-GPU box (never needed on an N-GPU node):
    # TCPCSUM_BENCH_SHARE_DEVICE=1 puts every rank on GPU 0.
    if os.environ.get("TCPCSUM_BENCH_SHARE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as tdist
        # no data-path collective: gloo (CPU) carries the barriers and the two reductions;
        # TCPCSUM_BENCH_BACKEND=nccl selects RCCL instead
        backend = os.environ.get("TCPCSUM_BENCH_BACKEND", "gloo")
        # gloo announces its connections on stdout; the one JSON line must stay alone there
        sys.stdout.flush()
        saved, null = os.dup(1), os.open(os.devnull, os.O_WRONLY)
        os.dup2(null, 1)
        try:
            if backend == "nccl":
                tdist.init_process_group("nccl", device_id=device)
            else:
                tdist.init_process_group(backend)
            tdist.barrier()
        finally:
            os.dup2(saved, 1)
            os.close(saved)
            os.close(null)
        dist = tdist
    rc, arch = tcp_amd.device_check()
    if rc != 0:
        raise SystemExit(f"bench.py: no usable gfx950 device ({rc}, '{arch}')")
    tcp_amd.set_tuning(args.max_blocks, args.unroll, args.shape, args.flags)

    if args.host_path_only:
        legs = {m: run_host_path(args.host_steps, min(args.warmup, 2), rank, world, local, dist, device, m)
                for m in ("pageable", "pinned")}
        if rank == 0:
            print(json.dumps({"metric": "GiB/s checksummed end-to-end (host memory in and out, PCIe-inclusive)",
                              "value": legs["pageable"]["GiB/s"], "unit": "GiB/s", "n_gpus": world,
                              "higher_is_better": True, "scaling": "weak", "dtype": "u16",
                              "data": "synthetic (SURVEY.md Appendix B generator)",
                              "ranks_share_one_gpu": os.environ.get("TCPCSUM_BENCH_SHARE_DEVICE") == "1",
                              "host_path": legs, "arch": arch}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return 0

    host_ctx = host_context(local) if (args.host_ctx_early and not args.no_host_path) else None
    host_first = None
    # The host leg runs after the device configs; --host-path-first runs it before them (A/B:
    # with the context's copies and kernels on one stream its rate no longer depends on the
    # order, DESIGN.md §7 "Order", profiles/r04_host_leg_order.jsonl).
    if args.host_path_first and not args.no_host_path:
        host_first = {m: run_host_path(args.host_steps, min(args.warmup, 2), rank, world, local, dist, device, m)
                      for m in ("pageable", "pinned")}
        torch.cuda.empty_cache()
    r, bufs, rot = run_config(args.config, args.steps, args.warmup, rank, world, dist, device, args.rotate,
                              streams=args.streams)
    L, cnt, batch_bytes, desc, check = r["L"], r["cnt"], r["batch_bytes"], r["desc"], r["check"]
    wall_max, kernel_ms, kernel_ms_max = r["wall_max"], r["kernel_ms"], r["kernel_ms_max"]
    stream = torch.cuda.current_stream()

    probe = None
    if world == 1 and not args.no_probe:
        pms = time_probe(bufs[:rot], batch_bytes, args.steps, device)
        probe = {"kernel": "k_probe<4> (read-only 16-B stream: one 4 KiB tile per wave, XCD order, as the plan)",
                 "avg_ms": round(pms, 5),
                 "GB/s": round((batch_bytes // 16) * 16 / (pms * 1e-3) / 1e9, 1),
                 "headline_kernel_over_probe": round(kernel_ms / pms, 4)}

    # the other single-GPU BASELINE configs (parity configs, reported beside the
    # headline: kernel rate vs the HBM roofline, digest check), N=1 only
    extra = {}
    if world == 1 and not args.no_other_configs:
        tcp_amd.set_tuning(0, 0, -1, 0)   # built-in launch shapes for the other configs
        # largest batch first: a 16 GiB batch allocated after smaller batches were freed runs
        # 2.43-2.47 ms per launch, 2.40 on memory no earlier batch used (tools/order_check.py,
        # profiles/r02_order_check.jsonl) — a property of the allocation, not of the kernel
        for cfg in sorted(CONFIGS, key=lambda c: -CONFIGS[c][0] * CONFIGS[c][1]):
            if cfg == args.config or (args.other and cfg not in args.other.split(",")):
                continue
            steps = max(10, min(args.steps, 200 if CONFIGS[cfg][1] < 4096 else 40))
            e, ebufs, erot = run_config(cfg, steps, min(args.warmup, 5), rank, world, dist, device)
            # the read-only probe over the same rotation, same box, same moment: the config's own
            # ceiling (for 64 B: a 64 MiB launch's ramp and drain bound the probe as well)
            epms = time_probe(ebufs[:erot], e["batch_bytes"], steps, device) if not args.no_probe else None
            del ebufs
            gbs = e["batch_bytes"] / (e["kernel_ms"] * 1e-3) / 1e9
            extra[cfg] = {"workload": e["desc"], "GiB/s": round(e["batch_bytes"] * steps / e["wall_max"] / (1 << 30), 2),
                          "kernel_avg_ms": round(e["kernel_ms"], 5), "achieved_GB/s": round(gbs, 1),
                          "roofline_frac": round(gbs / HBM_PEAK_GBS, 4), "steps": steps,
                          "window_ms_per_launch": round(e["window_ms"], 5),
                          "warmup_launches": e["warmup_launches"],
                          "rotating_batches": e["rot"], "digest_check": e["check"],
                          "traffic": load_traffic(cfg)}
            if epms:
                extra[cfg]["stream_probe"] = {"avg_ms": round(epms, 5),
                                              "GB/s": round(e["batch_bytes"] / (epms * 1e-3) / 1e9, 1),
                                              "kernel_over_probe": round(e["kernel_ms"] / epms, 4)}
            torch.cuda.empty_cache()
            if CONFIGS[cfg][1] < 4096:
                # small segments: the per-launch ramp is a large share of a launch; the same
                # batches pipelined over two streams (launch durations overlap, so the rate is
                # whole-run bytes / time, not bytes per launch duration)
                e2, ebufs, _ = run_config(cfg, steps, min(args.warmup, 5), rank, world, dist, device, streams=2)
                del ebufs
                gbs2 = e2["batch_bytes"] / (e2["kernel_ms"] * 1e-3) / 1e9
                extra[cfg]["two_streams"] = {
                    "GiB/s": round(e2["batch_bytes"] * steps / e2["wall_max"] / (1 << 30), 2),
                    "ms_per_launch_effective": round(e2["kernel_ms"], 5), "effective_GB/s": round(gbs2, 1),
                    "roofline_frac_effective": round(gbs2 / HBM_PEAK_GBS, 4), "digest_check": e2["check"]}
                torch.cuda.empty_cache()
                # the caller-facing form: K = 16 distinct batches in ONE launch
                # (tcpcsum_batch_uniform_multi_dev), the ramp and drain paid once per launch
                K = 16
                e3, ebufs, _ = run_config(cfg, max(5, steps // 8), min(args.warmup, 3), rank, world, dist, device,
                                          multi=K)
                del ebufs
                per_batch_ms = e3["kernel_ms"] / K
                gbs3 = e3["batch_bytes"] / (per_batch_ms * 1e-3) / 1e9
                extra[cfg]["multi_batch"] = {
                    "batches_per_launch": K, "api": "tcpcsum_batch_uniform_multi_dev",
                    "kernel_avg_ms_per_launch": round(e3["kernel_ms"], 5), "ms_per_batch": round(per_batch_ms, 5),
                    "GiB/s": round(e3["batch_bytes"] * K * max(5, steps // 8) / e3["wall_max"] / (1 << 30), 2),
                    "achieved_GB/s": round(gbs3, 1), "roofline_frac": round(gbs3 / HBM_PEAK_GBS, 4),
                    "digest_check": e3["check"], "traffic": load_traffic(cfg + "_multi")}
                torch.cuda.empty_cache()
        # the reference's own call site on wire packets (context.c:208): FILL and VERIFY in place,
        # on MTU packets and on the flush mix of control and data segments
        if not args.other or "wire" in args.other.split(","):
            extra["wire_1500"] = run_wire(max(10, min(args.steps, 100)), min(args.warmup, 5), device)
            torch.cuda.empty_cache()
        if not args.other or "wire_mix" in args.other.split(","):
            extra["wire_mix"] = run_wire_mix(max(10, min(args.steps, 100)), min(args.warmup, 5), device)
            torch.cuda.empty_cache()

    # end to end from host memory, every rank at once (PCIe and host DRAM bound; never `value`)
    host_path = None
    if not args.no_host_path and not args.host_path_first:
        del bufs
        torch.cuda.empty_cache()
        host_path = {m: run_host_path(args.host_steps, min(args.warmup, 2), rank, world, local, dist, device, m,
                                      ctx=host_ctx)
                     for m in ("pageable", "pinned")}

    if rank == 0:
        total_bytes = batch_bytes * world * args.steps
        value = total_bytes / wall_max / (1 << 30)
        achieved = batch_bytes / (kernel_ms * 1e-3) / 1e9   # rank 0's kernel, GB/s
        traffic = load_traffic(args.config)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (SURVEY.md Appendix B generator, generated in HBM before timing)",
            "config": {"workload": desc, "segments_per_gpu": cnt, "segment_bytes": L,
                       "parallelism": f"shard{world} (contiguous segment ranges, no collective)",
                       "rotating_batches": rot, "streams": args.streams, "arch": arch},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": ("profiles/traffic.json: HBM bytes per launch of this kernel from a "
                                            "separate rocprofv3 --pmc FETCH_SIZE pass (x2 gfx950 correction), "
                                            "committed, not measured in this run") if traffic else None,
                         "kernel": "tcpcsum::k_uniform (tcpcsum_batch_uniform_dev)",
                         "kernel_avg_ms": round(kernel_ms, 5), "kernel_avg_ms_max_rank": round(kernel_ms_max, 5),
                         "kernel_avg_over": "HIP events, launches 2..K of the timed window (the first waits on "
                                            "the host's enqueue)",
                         "window_ms_per_launch": round(r["window_ms"], 5),
                         "algorithmic_bytes_per_launch": batch_bytes},
            "digest_check": check,
        }
        if dist is not None:
            line["barrier_backend"] = dist.get_backend()
            line["ranks_share_one_gpu"] = os.environ.get("TCPCSUM_BENCH_SHARE_DEVICE") == "1"
        if probe:
            line["stream_probe"] = probe
        if extra:
            line["other_configs"] = extra
        if host_path or host_first:
            line["host_path"] = host_path or host_first
            line["host_path_order"] = "before the device configs" if host_first else "after the device configs"
        if seam:
            line["seam"] = seam
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
