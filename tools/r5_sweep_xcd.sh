# Round 5: uniform-kernel launch shapes under XCD-by-XCD tile order — per segment size, the
# current default (blocks 0, unroll 0) against one tile per wave (blocks 2^24) at unroll 1..8.
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
S="timeout -k 10 200 python3 -u tools/sweep.py --rounds 5 --steps 30 --blocks 0,16777216 --unrolls 0,1,2,4,8"
$S --config 64 --steps 200 > $O/t64.jsonl 2> $O/t64.err || exit $?
for L in 128 256 512 1499 1500 2048 3000 4096 6000; do
  $S --len $L > $O/t$L.jsonl 2> $O/t$L.err || exit $?
done
