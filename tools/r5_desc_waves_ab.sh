# Round 5: occupancy of the balanced ragged kernel (TCPCSUM_DESC_LB_WAVES measurement builds 7, 8)
# against the compiler's choice (6 waves per SIMD at 79 VGPRs), same process, shared inputs.
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
AB_ROUNDS=7 timeout -k 10 400 python3 -u tools/misc_lib_ab.py tcp_amd/ab/libtcpcsum_lbw7.so tcp_amd/ab/libtcpcsum_lbw8.so > $O/ab.jsonl 2> $O/ab.err
