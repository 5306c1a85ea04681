#!/bin/bash
# round 3: wire FILL line store (default) — every GPU test first, then the A/B timing three
# times (the two FILL stores must agree byte for byte every time)
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gputest_fill_line.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gputest_fill_line.log
if [ $rc -eq 0 ]; then
  for i in 1 2 3; do
    timeout -k 10 200 python tools/fill_line_ab.py --rounds 2 >> gpurun_out/fill_line_ab2.jsonl 2> gpurun_out/fill_line_ab.err || { echo "ab failed"; exit 1; }
  done
  echo ab ok
fi
