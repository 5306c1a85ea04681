# Round 5: read probe group shapes beside the headline kernel, and the write-back probe's
# shapes (one tile per wave in XCD order among them) beside the wire FILL.
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "probe" > $O/tests.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/sweep.py --config 1500 --rounds 5 --steps 30 --blocks 0 --unrolls 0 --probe --probe-shapes 0:0:-1,0:0:2,0:0:10,0:0:11,0:0:12 > $O/probe.jsonl 2> $O/probe.err || exit $?
PROBE_GRIDS=0,8192 PROBE_UNROLLS=0,1 ROUNDS=5 timeout -k 10 300 python3 -u tools/probe_rw_sweep.py > $O/rw.jsonl 2> $O/rw.err
