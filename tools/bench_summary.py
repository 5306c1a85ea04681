#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (tools/r6_runs.sh bench)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"],
      "kernel_ms", d["roofline"]["kernel_avg_ms"], "probe", d.get("stream_probe"), "digest", d["digest_check"])
for k, v in d.get("other_configs", {}).items():
    if k.startswith("wire"):
        print(k, {m: v[m].get("kernel_avg_ms", v[m].get("avg_ms")) for m in v if isinstance(v[m], dict)
                  and ("kernel_avg_ms" in v[m] or "avg_ms" in v[m])},
              {m: v[m] for m in v if m.endswith("_over_verify") or "_over_" in m}, "check", v.get("check"))
    else:
        print(k, v["kernel_avg_ms"], v["roofline_frac"], v.get("stream_probe"),
              (v.get("multi_batch") or {}).get("roofline_frac"))
for m, v in (d.get("host_path") or {}).items():
    print("host", m, v["GiB/s"], v.get("raw_pinned_h2d_GiB/s"), v["cpu_core_s_per_step_rank0"],
          v["cgroup_throttled_ms_per_rank"], v["digest_check"])
if "seam" in d:
    print("seam", json.dumps(d["seam"])[:1500])
cb = d.get("cpu_baseline") or {}
print("cpu", cb.get("value"), cb.get("throttle"))
