#!/bin/bash
# Round-end evidence (gpurun): GPU tests, smoke, default bench, N=2 rehearsal on one GPU
# (TCPCSUM_BENCH_SHARE_DEVICE=1: both ranks on cuda:0), rocprofv3 kernel trace of the headline.
set -e
O=gpurun_out/final
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 50 > $O/bench_n2_shared.json 2> $O/bench_n2.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/kt.err
echo done
