# Round 5: XCD order granularity (TCPCSUM_XCD_CHUNK measurement builds) against the product's
# contiguous eighths, then the probe without its workgroup barrier beside the kernel.
set -o pipefail
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "probe or uniform" > $O/tests.txt 2>&1 || exit $?
AB_ROUNDS=7 AB_LENS=3000 timeout -k 10 300 python3 -u tools/uniform_lib_ab.py tcp_amd/ab/libtcpcsum_chunk16.so tcp_amd/ab/libtcpcsum_chunk64.so tcp_amd/ab/libtcpcsum_chunk256.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err || exit $?
timeout -k 10 300 python3 -u tools/sweep.py --config 1500 --rounds 5 --steps 30 --blocks 0 --unrolls 0 --probe --probe-shapes 0:0:-1,0:0:2,0:0:3,0:1:-1 > $O/probe.jsonl 2> $O/probe.err
