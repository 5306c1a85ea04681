#!/bin/bash
# Lane-group wire kernel shapes across slot sizes, VERIFY and FILL (tools/wiresweep.py):
# auto (-1), 5 (8 x 12 chunks), 7 (8 x 4 chunks, more rounds), 8 (balanced).
set -e
for sp in "576 496" "1024 944" "1536 1456"; do
  set -- $sp
  SLOT=$1 PAYLOAD=$2 SHAPES=${SHAPES:--1,5,7,8} BLOCKS=${BLOCKS:-0,16384} UNROLLS=1 timeout -k 10 200 \
    python3 tools/wiresweep.py | grep -v round > gpurun_out/wire_mtu_sweep_$1.jsonl
done
