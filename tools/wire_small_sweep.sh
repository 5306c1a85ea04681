#!/bin/bash
# Wire shapes on small device-resident batches of MTU packets (1536-B slots).
set -e
O=gpurun_out/wsm
mkdir -p $O
for N in 1024 8192 32768; do
  N=$N SHAPES=-1,1,3,5,7 BLOCKS=0 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py > $O/n$N.jsonl 2>> $O/err
done
