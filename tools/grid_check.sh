#!/bin/bash
# New uniform default (blocks 0) against the previous caps (512 / 4096) at small and MTU sizes.
set -e
O=gpurun_out/grid_check
mkdir -p $O
for L in 64 100 128 200 256 576 1024 1500; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,512,4096 --unrolls 0 --rounds 5 --steps 20 > $O/len$L.jsonl 2>>$O/err
done
