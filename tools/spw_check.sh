#!/bin/bash
# Balanced ragged kernel with segments-per-wave sized by max_len: parity, sweep, A/B vs the previous build.
set -e
O=gpurun_out/spw
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -k "desc or balanced or fuzz" > $O/parity.log 2>&1
SIZES=1500,4096,9000,32768,65536 SHAPES=-1,4,5,6,8 ROUNDS=3 timeout -k 10 400 python3 tools/desc_sweep.py > $O/desc.jsonl 2> $O/err
timeout -k 10 300 python3 tools/lb_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/lb_ab.jsonl 2>> $O/err
