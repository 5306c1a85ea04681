#!/usr/bin/env python3
"""Does the 64 KiB config's rate depend on what ran before it in the process?

bench.py reports the 64 KiB config after the 1500-B and 64-B configs (2.47 ms per
launch on MI355X) while a process that runs it alone measures 2.39-2.40 ms. This
runs bench.run_config in several orders in separate processes and prints one
line per (order, config)."""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ORDERS = [["64k"], ["1500", "64k"], ["64", "64k"], ["64", "64s2", "64k"], ["1500", "64", "64s2", "64k"],
          ["64k", "64k"]]


def child(order):
    import torch
    import bench
    dev = torch.device("cuda:0")
    keep = []
    for i, cfg in enumerate(order):
        streams = 2 if cfg.endswith("s2") else 1
        name = cfg[:-2] if streams == 2 else cfg
        steps = 200 if name != "64k" else 40
        r, bufs, _ = bench.run_config(name, steps, 5, 0, 1, None, dev, streams=streams)
        if i == 0 and name == "1500":
            keep.append(bufs)          # bench.py keeps the headline buffers alive
        else:
            del bufs
        torch.cuda.empty_cache()
        print(json.dumps({"order": "+".join(order), "step": i, "config": cfg, "kernel_ms": round(r["kernel_ms"], 5),
                          "check": r["check"]}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(sys.argv[1].split("+"))
    else:
        for o in ORDERS:
            subprocess.run([sys.executable, os.path.abspath(__file__), "+".join(o)], check=True, timeout=300)
