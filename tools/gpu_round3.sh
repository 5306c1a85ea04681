timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gputest_r3b.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/gputest_r3b.log | grep -E "passed|failed|FAILED|Error" 
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 6 > gpurun_out/bench_r3b.json 2> gpurun_out/bench_r3b.err; echo "bench rc=$?"
fi
