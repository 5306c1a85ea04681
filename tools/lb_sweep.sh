set -e
for cfg in "0,0,9,0 0,0,8,0" "1024,0,8,0 1024,0,7,0" "2048,0,8,0 2048,0,7,0" "16384,0,8,0 16384,0,7,0"; do
  set -- $cfg
  LB_HEAD_WIRE=$1 LB_HEAD_DESC=$2 timeout -k 10 120 python3 tools/lb_ab.py tcp_amd/ab/libtcpcsum_r02a.so > gpurun_out/lbsweep_$1.jsonl 2>>gpurun_out/lbsweep.err
done
