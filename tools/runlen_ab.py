#!/usr/bin/env python3
"""Why the driver's short bench run reads the 64-B config slower than a 200-step run
(VERDICT r5 weak #2 / next #1). One process, fresh allocations for every variant:

  per_launch   32 fresh 64 MiB rotations (as bench.py allocates them), then 3 passes over all 32
               with a HIP event between launches: pass 1 is every batch's first read after the
               generator wrote it, passes 2-3 are repeat reads. A clock ramp shows as a slope
               inside pass 1; a first-read cost shows as pass 1 uniformly above passes 2-3.
  probe_first  the same for the read-only probe, on fresh rotations it has to read first.
  bench_forms  bench.py's own run_config / time_probe at (steps, warmup) = (20, 5) as the driver
               runs it, (200, 10), and (20, 5) after one untimed launch over every rotation.

Prints one JSON object per measurement. Config via RUNLEN_CONFIGS (default "64,1500").
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import tcp_amd  # noqa: E402
import bench  # noqa: E402


def fresh(config, device, rot=None):
    per_gpu, L, _ = bench.CONFIGS[config]
    nbytes = per_gpu * L
    rot = rot or max(1, -(-(2 << 30) // nbytes))
    bufs, sss = [], []
    for r in range(rot):
        d = torch.empty(nbytes, dtype=torch.uint8, device=device)
        s = torch.empty(per_gpu, dtype=torch.int32, device=device)
        tcp_amd.synth_fill(d, r * per_gpu * L, nbytes)
        tcp_amd.synth_pseudo(s, 0, per_gpu, L)
        bufs.append(d)
        sss.append(s)
    torch.cuda.synchronize()
    return L, per_gpu, nbytes, bufs, sss


def per_launch(config, device, what, passes=3):
    L, n, nbytes, bufs, sss = fresh(config, device)
    out = torch.empty(n, dtype=torch.int16, device=device)
    pout = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=device)
    st = torch.cuda.current_stream()
    launches = passes * len(bufs)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
    for e in ev:
        e.record(st)
    torch.cuda.synchronize()
    ev[0].record(st)
    for k in range(launches):
        r = k % len(bufs)
        if what == "kernel":
            tcp_amd.batch_uniform(bufs[r], L, L, n, sss[r], out=out, stream=st)
        else:
            tcp_amd.stream_probe(bufs[r], (nbytes // 16) * 16, pout, stream=st, tune=(0, 0, -1, 0))
        ev[k + 1].record(st)
    torch.cuda.synchronize()
    us = [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(launches)]
    R = len(bufs)
    rows = {f"pass{p + 1}": us[p * R:(p + 1) * R] for p in range(passes)}
    summ = {k: {"median_us": round(statistics.median(v), 2), "first4_us": [round(x, 2) for x in v[:4]],
                "last4_us": [round(x, 2) for x in v[-4:]]} for k, v in rows.items()}
    del bufs, sss
    torch.cuda.empty_cache()
    return {"exp": "per_launch", "config": config, "what": what, "rotations": R, **summ}


def bench_form(config, device, steps, warmup, prewarm):
    """bench.run_config as the bench calls it; prewarm: one untimed launch over every rotation first
    (done by running run_config's own warm-up over them: warmup = rot + warmup)."""
    per_gpu, L, _ = bench.CONFIGS[config]
    rot = max(1, -(-(2 << 30) // (per_gpu * L)))
    w = warmup + (rot if prewarm else 0)
    r, bufs, rot = bench.run_config(config, steps, w, 0, 1, None, device)
    pms = bench.time_probe(bufs[:rot], r["batch_bytes"], steps, device)
    del bufs
    torch.cuda.empty_cache()
    return {"exp": "bench_form", "config": config, "steps": steps, "warmup": warmup, "prewarm_all_rotations": prewarm,
            "kernel_us": round(r["kernel_ms"] * 1e3, 2), "probe_us": round(pms * 1e3, 2),
            "kernel_over_probe": round(r["kernel_ms"] / pms, 4), "check": r["check"]}


def cpu_enqueue(config, device, launches=200):
    """Host cost of one launch from Python: the GPU is held busy by a sleep kernel while the
    launches are enqueued, so the time is the CPU's alone; then the GPU time of the same launches
    (events around them, queued behind the sleep: no host gap inside)."""
    L, n, nbytes, bufs, sss = fresh(config, device)
    out = torch.empty(n, dtype=torch.int16, device=device)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(len(bufs)):   # every rotation read once
        tcp_amd.batch_uniform(bufs[r], L, L, n, sss[r], out=out, stream=st)
    torch.cuda.synchronize()
    import time
    torch.cuda._sleep(int(2e8))   # ~ 100 ms at 2 GHz
    e0.record(st)
    t0 = time.perf_counter()
    for k in range(launches):
        r = k % len(bufs)
        tcp_amd.batch_uniform(bufs[r], L, L, n, sss[r], out=out, stream=st)
    t1 = time.perf_counter()
    e1.record(st)
    torch.cuda.synchronize()
    del bufs, sss
    torch.cuda.empty_cache()
    return {"exp": "cpu_enqueue", "config": config, "launches": launches,
            "host_us_per_launch": round((t1 - t0) / launches * 1e6, 2),
            "gpu_us_per_launch_queued": round(e0.elapsed_time(e1) / launches * 1e3, 2)}


def first_read_parts(config, device, variant):
    """One pass over 32 fresh rotations, queued behind a sleep kernel (no host gaps), per-launch
    GPU time. variant: "base" (start-value arrays, nothing touched first), "scalar" (one scalar
    start value: no array read), "ss_warm" (every start-value array read once first),
    "data_warm" (every data batch read once first by the probe), "both_warm"."""
    L, n, nbytes, bufs, sss = fresh(config, device)
    out = torch.empty(n, dtype=torch.int16, device=device)
    pout = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=device)
    st = torch.cuda.current_stream()
    acc = torch.zeros(1, dtype=torch.int64, device=device)
    if variant in ("ss_warm", "both_warm"):
        for s in sss:
            acc += s.sum()
    if variant in ("data_warm", "both_warm"):
        for d in bufs:
            tcp_amd.stream_probe(d, (nbytes // 16) * 16, pout, stream=st, tune=(0, 0, -1, 0))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(5e7))
    e0.record(st)
    for r in range(len(bufs)):
        tcp_amd.batch_uniform(bufs[r], L, L, n, 7 if variant == "scalar" else sss[r], out=out, stream=st)
    e1.record(st)
    torch.cuda.synchronize()
    R = len(bufs)
    del bufs, sss
    torch.cuda.empty_cache()
    return {"exp": "first_read_parts", "config": config, "variant": variant, "rotations": R,
            "gpu_us_per_launch": round(e0.elapsed_time(e1) / R * 1e3, 2)}


def main():
    if os.environ.get("RUNLEN_ONLY") == "parts" or "--parts" in sys.argv:
        device = torch.device("cuda", 0)
        for rep in range(3):
            for v in ("base", "scalar", "ss_warm", "data_warm", "both_warm"):
                print(json.dumps({**first_read_parts("64", device, v), "rep": rep}), flush=True)
        return
    device = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    rc, arch = tcp_amd.device_check()
    assert rc == 0, arch
    for config in os.environ.get("RUNLEN_CONFIGS", "64,1500").split(","):
        print(json.dumps(cpu_enqueue(config, device)), flush=True)
        for rep in range(2):
            for what in ("kernel", "probe"):
                print(json.dumps({**per_launch(config, device, what), "rep": rep}), flush=True)
            for steps, warmup, pre in ((20, 5, False), (200, 10, False), (20, 5, True)):
                print(json.dumps({**bench_form(config, device, steps, warmup, pre), "rep": rep}), flush=True)


if __name__ == "__main__":
    main()
