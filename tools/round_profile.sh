#!/bin/bash
# Round-end evidence on one MI355X (run through gpurun): GPU tests, smoke, the
# default bench line, and rocprofv3 summaries of the headline kernel — kernel
# trace (average duration must agree with bench.py's HIP events) and a separate
# FETCH_SIZE pass (traffic) — plus WRITE_SIZE of the wire FILL. Outputs under
# gpurun_out/round/; copy what is judged into profiles/.
set -e
R=${1:-r02}
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline --probe"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $B > $O/bench_under_rocprof.json 2> $O/kt.err
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- $B > $O/pmc_fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_wire_write -o p -- python3 tools/fillbench.py > $O/pmc_wire_write.log 2>&1
echo done
