#!/bin/bash
# Wire shape 10 (window chunks through LDS) against the lane-group defaults.
set -e
O=gpurun_out/lds
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread -k "ipv4 or fuzz or ptrs" > $O/parity.log 2>&1
for S in 1536 1024 2048; do
  SLOT=$S SHAPES=-1,5,7,10 BLOCKS=0 UNROLLS=1 timeout -k 10 300 python3 tools/wiresweep.py > $O/slot$S.jsonl 2>> $O/err
done
