# Round 5: the XCD-order plan at HEAD against the previous build (tcp_amd/ab/libtcpcsum_prev.so):
# GPU tests, uniform sizes, wire workloads, tx_build and ragged batches, then the default bench.
set -o pipefail
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1 || exit $?
AB_ROUNDS=5 AB_LENS=128,256,1024,2048,3000,4096,8192,9000,12300,99,577,1499,3001 timeout -k 10 400 python3 -u tools/uniform_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/ab.jsonl 2> $O/ab.err || exit $?
timeout -k 10 300 python3 -u tools/wire_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/wire_ab.jsonl 2> $O/wire_ab.err || exit $?
timeout -k 10 300 python3 -u tools/misc_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/misc_ab.jsonl 2> $O/misc_ab.err || exit $?
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err
