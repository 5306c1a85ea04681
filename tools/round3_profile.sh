#!/bin/bash
# Round-3 evidence on one MI355X (through gpurun): rocprofv3 kernel trace of the
# headline bench (its average must agree with bench.py's HIP events), FETCH_SIZE
# of the headline kernel, FETCH/WRITE_SIZE of the 64-B multi-batch launch, and
# WRITE_SIZE / FETCH_SIZE of the wire FILL stores (2-byte vs line vs VERIFY).
# Every pass is its own run (rocprofv3 does not split counters over passes).
O=gpurun_out/r3prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline --probe"
run() { echo "== $1"; shift; "$@" || { echo "failed: $?"; exit 1; }; }
run kt timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $B > $O/bench_under_rocprof.json 2> $O/kt.err
run fetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- $B > $O/pmc_fetch.log 2>&1
M="python3 tools/multi_sweep.py --ks 16 --unrolls 4 --grids 0 --rounds 1 --steps 10"
run mfetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_multi_fetch -o p -- $M > $O/pmc_multi_fetch.log 2>&1
run mwrite timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_multi_write -o p -- $M > $O/pmc_multi_write.log 2>&1
W="python3 tools/wire_fill_pmc.py"
run wwrite timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_wire_write -o p -- $W > $O/pmc_wire_write.log 2>&1
run wfetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_wire_fetch -o p -- $W > $O/pmc_wire_fetch.log 2>&1
run wkt timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_wire -o k -- $W > $O/kt_wire.log 2>&1
echo done
