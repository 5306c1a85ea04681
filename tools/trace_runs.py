#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (CSV) as runs of consecutive launches of one kernel:
count, median / first / last duration, median gap between launches, span per launch.

  python tools/trace_runs.py <kernel_trace.csv> [min_run=5]  -> one JSON object per run
"""
import csv
import json
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    min_run = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
    runs = []
    for s, e, k in seq:
        if runs and runs[-1][0] == k:
            runs[-1][1].append((s, e))
        else:
            runs.append([k, [(s, e)]])
    for k, launches in runs:
        if len(launches) < min_run:
            continue
        d = [(e - s) / 1e3 for s, e in launches]
        gaps = [(launches[i + 1][0] - launches[i][1]) / 1e3 for i in range(len(launches) - 1)]
        print(json.dumps({"kernel": k, "launches": len(d), "median_us": round(statistics.median(d), 2),
                          "mean_us": round(statistics.mean(d), 2), "first3_us": [round(x, 2) for x in d[:3]],
                          "last3_us": [round(x, 2) for x in d[-3:]], "median_gap_us": round(statistics.median(gaps), 2),
                          "span_per_launch_us": round((launches[-1][1] - launches[0][0]) / 1e3 / len(d), 2)}))


if __name__ == "__main__":
    main()
