#!/bin/bash
# Wire defaults after the size-class rule: parity, then the default shape per slot size.
set -e
O=gpurun_out/wdef
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread -k "ipv4 or fuzz or ptrs" > $O/parity.log 2>&1
for S in 1536 2048 3072 4608 9216; do
  SLOT=$S SHAPES=-1,1,7 BLOCKS=0 UNROLLS=1 timeout -k 10 300 python3 tools/wiresweep.py > $O/slot$S.jsonl 2>> $O/err
done
