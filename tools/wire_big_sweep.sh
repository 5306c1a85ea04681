#!/bin/bash
# Wire lane-group shapes on packets between the MTU and jumbo sizes (slots 2-9 KiB).
set -e
O=gpurun_out/wbig
mkdir -p $O
for S in 2048 3072 4608 9216; do
  SLOT=$S SHAPES=-1,1,2,4,7 BLOCKS=0 UNROLLS=1,2 timeout -k 10 300 python3 tools/wiresweep.py > $O/slot$S.jsonl 2>> $O/err
done
