#!/bin/bash
# Split-segment kernel (shape 13) vs shape 9, second pass: jumbo / byte-granular / aligned mid sizes.
set -e
O=gpurun_out/split2
mkdir -p $O
for L in 9000 8999 12301 16384 24576 49152 65536 65532; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --shapes 9,13 --blocks 0 --unrolls 0,1,2 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
done
timeout -k 10 300 python3 tools/sweep.py --config 64k --shapes 9,13 --blocks 0,1024,4096 --unrolls 0,2 --rounds 3 --steps 5 > $O/cfg64k.jsonl 2>>$O/err
