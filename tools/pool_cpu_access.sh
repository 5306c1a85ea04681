#!/usr/bin/env bash
# The interposer's arena (TCPCSUM_PRELOAD_POOL) as CPU memory: the reference's CPU checksum over
# the out-buffers and a recvmmsg + CPU verify over the in-buffers, arena vs malloc, GPU seams off.
mkdir -p gpurun_out/r5
P=$PWD/tcp_amd/libtcpcsum_preload.so
for rep in 1 2; do
  for pool in 0 mmsg_bench; do
    timeout -k 10 120 env LD_PRELOAD=$P TCPCSUM_PRELOAD_TX=off TCPCSUM_PRELOAD_RX=off TCPCSUM_PRELOAD_STATS=1 TCPCSUM_PRELOAD_POOL=$pool tools/mmsg_bench cpu 300 > gpurun_out/r5/pc_cpu_${pool}_$rep.json 2> gpurun_out/r5/pc_cpu_${pool}_$rep.err || exit $?
    timeout -k 10 120 env LD_PRELOAD=$P TCPCSUM_PRELOAD_TX=off TCPCSUM_PRELOAD_RX=off TCPCSUM_PRELOAD_STATS=1 TCPCSUM_PRELOAD_POOL=$pool tools/mmsg_bench rxcpu 300 > gpurun_out/r5/pc_rxcpu_${pool}_$rep.json 2> gpurun_out/r5/pc_rxcpu_${pool}_$rep.err || exit $?
    echo "pool=$pool rep=$rep cpu: $(python3 -c "import json; d=json.load(open('gpurun_out/r5/pc_cpu_${pool}_$rep.json')); print(d['median_us'], d['checks_match_cpu'])") $(grep -o 'served=[0-9]*' gpurun_out/r5/pc_cpu_${pool}_$rep.err) rxcpu: $(python3 -c "import json; d=json.load(open('gpurun_out/r5/pc_rxcpu_${pool}_$rep.json')); print(d['median_us'], d['verified_last'])") $(grep -o 'served=[0-9]*' gpurun_out/r5/pc_rxcpu_${pool}_$rep.err)"
  done
done
