# Round 5: XCD order in the ragged and long-segment kernels — balanced tile sizes on ragged
# batches, the ragged default against the previous build, the 64 KiB config's grids, and
# byte-granular long segments.
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py > $O/tests.txt 2>&1 || exit $?
SIZES=0,1500 SHAPES=7,8 UNROLLS=0,2,4,8 ROUNDS=5 timeout -k 10 300 python3 -u tools/desc_sweep.py > $O/desc.jsonl 2> $O/desc.err || exit $?
AB_ROUNDS=7 timeout -k 10 300 python3 -u tools/misc_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/misc_ab.jsonl 2> $O/misc_ab.err || exit $?
timeout -k 10 300 python3 -u tools/sweep.py --config 64k --rounds 5 --steps 5 --blocks 0,16777216 --unrolls 0 --shapes=-1,13 > $O/s64k.jsonl 2> $O/s64k.err || exit $?
AB_ROUNDS=5 AB_LENS=12301,20001 timeout -k 10 300 python3 -u tools/uniform_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/ab.jsonl 2> $O/ab.err
