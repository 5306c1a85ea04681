#!/bin/bash
# e2e_multi.sh — the end-to-end (host memory) leg of bench.py on N ranks at once, one context
# per GPU (bench.run_host_path): pageable and pinned shards of the global 1500-B config, every
# rank's results checked against its Appendix B digest, one JSON line.
#   bash tools/e2e_multi.sh N [steps]      (N ranks, one per GPU)
#   TCPCSUM_BENCH_SHARE_DEVICE=1 bash tools/e2e_multi.sh 2   (rehearsal: every rank on GPU 0)
N=${1:-2}
STEPS=${2:-5}
python3 bench.py --gpus "$N" --host-path-only --host-steps "$STEPS" --warmup 2
