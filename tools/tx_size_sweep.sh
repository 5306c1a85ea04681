#!/bin/bash
# Segment builder shapes across payload sizes (pure ACK .. jumbo).
set -e
O=gpurun_out/txs
mkdir -p $O
for L in 0 40 536 1456 4000 8956; do
  TX_LEN=$L TX_SHAPES=-1,0,1,2,3,4 TX_BLOCKS=32768 TX_UNROLLS=1 timeout -k 10 300 python3 tools/txbench.py --sweep > $O/len$L.jsonl 2>> $O/err
done
