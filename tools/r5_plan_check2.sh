# Round 5: after keeping block order where XCD order did not win — kernel parity tests, the A/Bs
# against tcp_amd/ab/libtcpcsum_prev.so, the probe's tile sizes, then the headline bench with its
# rocprofv3 kernel trace and FETCH_SIZE pass.
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py tests/test_gpu_graph.py tests/test_gpu_multi.py > $O/tests.txt 2>&1 || exit $?
AB_ROUNDS=5 AB_LENS=8192,12300,1499 timeout -k 10 300 python3 -u tools/uniform_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/ab.jsonl 2> $O/ab.err || exit $?
timeout -k 10 300 python3 -u tools/wire_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/wire_ab.jsonl 2> $O/wire_ab.err || exit $?
AB_ROUNDS=7 timeout -k 10 300 python3 -u tools/misc_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/misc_ab.jsonl 2> $O/misc_ab.err || exit $?
timeout -k 10 300 python3 -u tools/sweep.py --config 1500 --rounds 5 --steps 30 --blocks 0 --unrolls 0 --probe --probe-shapes 0:0,16777216:0,512:2,8192:1,16777216:1,16777216:2 > $O/probe.jsonl 2> $O/probe.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_h -o fetch -- python3 bench.py --steps 50 --no-other-configs --no-host-path --no-cpu-baseline > $O/pmc_h.json 2> $O/pmc_h.err
