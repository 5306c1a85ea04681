#!/bin/bash
# Balanced kernels: per-lane sums for tiles of small segments, against the previous build.
set -e
O=gpurun_out/lane
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
timeout -k 10 300 python3 tools/lb_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/lb_ab.jsonl 2> $O/lb_ab.err
