# Round 5 final rehearsal (one run): every GPU test, smoke(), the default bench, the bench under
# rocprofv3 --kernel-trace --stats, and the headline FETCH_SIZE pass.
set -o pipefail
O=${R5_OUT:-gpurun_out/r5final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gputest.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_h -o fetch -- python3 bench.py --steps 50 --no-other-configs --no-host-path --no-cpu-baseline > $O/pmc_h.json 2> $O/pmc_h.err
