# Round 5: the fused builder's grid — its default (32768 workgroups, looping) against one tile per
# wave (XCD order), interleaved, at four payload sizes.
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
for L in 1456 536 200 3000; do
  TX_LEN=$L TX_ROUNDS=5 TX_SHAPES=-1 TX_BLOCKS=32768,16777216 TX_UNROLLS=0 timeout -k 10 200 python3 -u tools/txbench.py --sweep > $O/tx$L.jsonl 2> $O/tx$L.err || exit $?
done
