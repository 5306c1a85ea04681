set -e
for sp in "768 688" "896 816"; do
  set -- $sp
  SLOT=$1 PAYLOAD=$2 SHAPES=8,7 BLOCKS=0,16384 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py | grep -v round > gpurun_out/wire_mtu_sweep_$1.jsonl
done
