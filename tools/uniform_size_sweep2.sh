#!/bin/bash
# Uniform 6-8 KiB segments: shape 8 (64 lanes x 8 chunks) against one wave (9) and four waves (13) per segment.
set -e
O=gpurun_out/usz2
mkdir -p $O
for L in 6400 7000 7600 8000 8192; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --shapes=-1,9,13 --blocks 0 --unrolls 0,1 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
done
