#!/bin/bash
# Split-segment kernel (shape 13: four waves per segment) against the
# one-wave-per-segment kernel (shape 9) on long uniform segments.
set -e
O=gpurun_out/split
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "forced_shapes or long_segments or two_fold or all_unrolls" > $O/parity.log 2>&1
for L in 12300 20004 32768 65536 131072; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --shapes 9,13 --blocks 0 --unrolls 0,2,4,8 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
done
timeout -k 10 300 python3 tools/sweep.py --config 64k --shapes 9,13 --blocks 0 --unrolls 0,2,4,8 --rounds 3 --steps 5 > $O/cfg64k.jsonl 2>>$O/err
