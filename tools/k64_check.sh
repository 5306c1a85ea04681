#!/bin/bash
# 64 KiB config: why bench.py (2.47 ms) and the sweep (2.40 ms) differ — steps, warmup, shape.
set -e
O=gpurun_out/k64
mkdir -p $O
B="python3 bench.py --config 64k --no-cpu-baseline --no-other-configs"
for s in 5 40; do
  timeout -k 10 120 $B --steps $s --warmup 3 > $O/bench_s$s.json 2>>$O/err
  timeout -k 10 120 $B --steps $s --warmup 3 --shape 9 > $O/bench_s${s}_shape9.json 2>>$O/err
done
timeout -k 10 200 python3 tools/sweep.py --config 64k --shapes 9,13 --blocks 0 --unrolls 0 --rounds 2 --steps 40 > $O/sweep_s40.jsonl 2>>$O/err
