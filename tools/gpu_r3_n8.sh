#!/bin/bash
# round 3: the wire FILL change under every GPU test and the A/B, then an N=8 rehearsal of
# bench.py on one GPU (all eight ranks share it; every rank checks its 8Mx1500 shard digest)
bash tools/gpu_r3_fill.sh || exit 1
TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 8 --steps 5 --warmup 2 --no-other-configs > gpurun_out/bench_n8_shared.json 2> gpurun_out/bench_n8_shared.err
echo "n8 rc=$?"; cat gpurun_out/bench_n8_shared.json | cut -c1-400
