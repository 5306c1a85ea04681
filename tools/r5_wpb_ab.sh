# Round 5: waves per workgroup of the uniform kernel (TCPCSUM_UNIFORM_WPB measurement builds 1, 2)
# against the product's 4, same process.
set -o pipefail
O=gpurun_out/r5m
mkdir -p $O
AB_ROUNDS=7 AB_LENS=256,1024,3000 timeout -k 10 400 python3 -u tools/uniform_lib_ab.py tcp_amd/ab/libtcpcsum_wpb1.so tcp_amd/ab/libtcpcsum_wpb2.so > $O/ab.jsonl 2> $O/ab.err
