#!/bin/bash
# Segment builder: (16,2) vs (32,3) lane groups between 256 B and 1.2 KiB payloads.
set -e
O=gpurun_out/txs2
mkdir -p $O
for L in 256 536 768 1024 1200; do
  TX_LEN=$L TX_SHAPES=2,1,2,1 TX_BLOCKS=32768 TX_UNROLLS=1 timeout -k 10 300 python3 tools/txbench.py --sweep > $O/len$L.jsonl 2>> $O/err
done
