#!/bin/bash
# Balanced wire kernel on 64K-128K-packet batches: auto (>= 4096 wave tiles) vs forced 64-packet tiles.
set -e
O=gpurun_out/wlbs
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread -k "ipv4 or fuzz or ptrs" > $O/parity.log 2>&1
for N in 65536 131072; do
  N=$N SLOT=84 PAYLOAD=40 SHAPES=-1,8,0 BLOCKS=0 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py > $O/s84_n$N.jsonl 2>> $O/err
  N=$N SLOT=576 PAYLOAD=496 SHAPES=-1,8,7 BLOCKS=0 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py > $O/s576_n$N.jsonl 2>> $O/err
done
