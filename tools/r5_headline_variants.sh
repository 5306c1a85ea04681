# Round 5: headline tile plan against neighbouring (grid-stride) grids,
# plus the wire workloads and ragged batches at HEAD against the previous build.
set -o pipefail
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 300 python3 -u tools/sweep.py --config 1500 --rounds 7 --steps 30 --blocks 0,65536,32768 --unrolls 0 > $O/s1500_flags.jsonl 2> $O/s1500_flags.err || exit $?
timeout -k 10 300 python3 -u tools/wire_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/wire_ab.jsonl 2> $O/wire_ab.err || exit $?
AB_ROUNDS=7 timeout -k 10 300 python3 -u tools/misc_lib_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/misc_ab.jsonl 2> $O/misc_ab.err
