#!/bin/bash
# gpu_runs.sh — the GPU experiments behind DESIGN.md, one function each, run on an MI355X
# box through gpurun:  /usr/local/graft/bin/gpurun -- bash tools/gpu_runs.sh <name>
# (`bash tools/gpu_runs.sh` alone lists them). Outputs go under gpurun_out/; the
# summaries judged are copied into profiles/. Every GPU step has its own time limit.

# round 4, first pass: every GPU test in one process (no child isolation left), the smoke, the
# wire A/B against the round-3 build (asm stores + spilled FILL) and the host-path / seam sweeps
# (wall time and CPU time per batch). Stops at the first GPU step that faults, aborts or times out.
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
gpu_r4_first() {
(
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r4_gputest1.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4_gputest1.log | tail -2; grep FAILED gpurun_out/r4_gputest1.log | head -20
  ok_rc $rc || exit $rc
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 gpurun_out/r4_smoke.log
  ok_rc $rc || exit $rc
  timeout -k 10 300 python -u tools/wire_lib_ab.py tcp_amd/ab/libtcpcsum_wire_r3.so > gpurun_out/r4_wire_ab_r3.jsonl 2> gpurun_out/r4_wire_ab_r3.err; rc=$?
  echo "wire ab rc=$rc"; ok_rc $rc || exit $rc
  timeout -k 10 500 python -u tools/e2e.py > gpurun_out/r4_e2e.jsonl 2> gpurun_out/r4_e2e.err; rc=$?
  echo "e2e rc=$rc"; ok_rc $rc || exit $rc
  timeout -k 10 300 bash tools/e2e_multi.sh 1 > gpurun_out/r4_e2e_multi_n1.json 2> gpurun_out/r4_e2e_multi_n1.err; rc=$?
  echo "e2e n1 rc=$rc"; ok_rc $rc || exit $rc
  TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 300 bash tools/e2e_multi.sh 2 > gpurun_out/r4_e2e_multi_n2_shared.json 2> gpurun_out/r4_e2e_multi_n2_shared.err; rc=$?
  echo "e2e n2 shared rc=$rc"
)
}

# round 4: GPU tests, then the host-path / seam sweep again (wait modes, copy threads)
gpu_r4_e2e() {
(
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4_gputest2.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4_gputest2.log | tail -2; grep FAILED gpurun_out/r4_gputest2.log | head -20
  ok_rc $rc || exit $rc
  timeout -k 10 500 python -u tools/e2e.py > gpurun_out/r4_e2e_${TAG:-b}.jsonl 2> gpurun_out/r4_e2e_${TAG:-b}.err; rc=$?
  echo "e2e rc=$rc"
)
}

# round 4: the wire FILL block-store variants (128-B line vs 64-B block vs 2-byte) — parity of the
# store variants first, then the interleaved A/B, then the e2e sweep
gpu_r4_fillhalf() {
(
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "window_and_store or ipv4" > gpurun_out/r4_fillhalf_parity.log 2>&1; rc=$?
  echo "parity rc=$rc"; grep -E "passed|failed" gpurun_out/r4_fillhalf_parity.log | tail -1
  ok_rc $rc || exit $rc
  timeout -k 10 300 python -u tools/fill_line_ab.py --rounds 5 > gpurun_out/r4_fill_half_ab.jsonl 2> gpurun_out/r4_fill_half_ab.err; rc=$?
  echo "ab rc=$rc"; ok_rc $rc || exit $rc
  timeout -k 10 500 python -u tools/e2e.py > gpurun_out/r4_e2e_b.jsonl 2> gpurun_out/r4_e2e_b.err; rc=$?
  echo "e2e rc=$rc"
)
}

# round 4: the default bench line once (new host_path leg at N=1) and N=2 with both ranks on one GPU
gpu_r4_bench() {
(
  timeout -k 10 500 python3 bench.py > gpurun_out/r4_bench_${TAG:-a}.json 2> gpurun_out/r4_bench_${TAG:-a}.err; rc=$?
  echo "bench rc=$rc"; ok_rc $rc || exit $rc
  TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 50 > gpurun_out/r4_bench_n2_shared_${TAG:-a}.json 2> gpurun_out/r4_bench_n2_shared_${TAG:-a}.err; rc=$?
  echo "bench n2 rc=$rc"
)
}

# round 4: NUMA placement of the host-path leg — the bench's thread affinity (first touch) and
# the context's copy-thread pinning on / off, interleaved twice, N=1
gpu_r4_numa() {
(
  for rep in 1 2; do
    for a in 1 0; do
      for n in 1 0; do
        TCPCSUM_BENCH_HOST_NUMA=$a TCPCSUM_HOST_NUMA=$n timeout -k 10 200 python3 bench.py --host-path-only --host-steps 10 > gpurun_out/r4_numa_a${a}_n${n}_rep$rep.json 2>> gpurun_out/r4_numa.err; rc=$?
        echo "a=$a n=$n rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/r4_numa_a${a}_n${n}_rep$rep.json'))['host_path']; print(d['pageable']['GiB/s'], d['pinned']['GiB/s'], d['pageable']['numa_node_rank0'], d['pageable']['cpu_core_s_per_step_rank0'])")"
        ok_rc $rc || exit $rc
      done
    done
  done
  lscpu | grep -i numa >> gpurun_out/r4_numa_topology.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r4_numa_topology.txt 2>/dev/null; true
)
}

# round 4: GPU tests after the NUMA staging change, then the host-path leg twice (NUMA nodes reported)
gpu_r4_numa2() {
(
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4_gputest3.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4_gputest3.log | tail -2; grep FAILED gpurun_out/r4_gputest3.log | head -20
  ok_rc $rc || exit $rc
  for rep in 1 2; do
    timeout -k 10 200 python3 bench.py --host-path-only --host-steps 10 > gpurun_out/r4_numa2_rep$rep.json 2>> gpurun_out/r4_numa2.err; rc=$?
    echo "rep $rep rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_numa2_rep$rep.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m]['numa_node_rank0'], d[m]['staging_numa_node_rank0'], d[m]['data_numa_node_rank0']) for m in d})")"
    ok_rc $rc || exit $rc
  done
)
}

# round 4: N=8 rehearsal of the whole bench (device headline + the host-memory leg on every rank)
# with all eight ranks on the one GPU of this box
gpu_r4_n8() {
(
  TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 8 --steps 5 --warmup 2 > gpurun_out/r4_bench_n8_shared.json 2> gpurun_out/r4_bench_n8_shared.err; rc=$?
  echo "n8 rc=$rc"; cut -c1-300 gpurun_out/r4_bench_n8_shared.json
)
}

# round 4, final rehearsal at HEAD: every GPU test, the smoke, the default bench line, and a
# rocprofv3 kernel trace of the headline (its average must agree with the line's HIP events)
gpu_r4_final() {
(
  O=gpurun_out/r4final
  mkdir -p $O
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -1; grep FAILED $O/gputest.log | head
  ok_rc $rc || exit $rc
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -1 $O/smoke.log; ok_rc $rc || exit $rc
  timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err; rc=$?
  echo "bench rc=$rc"; ok_rc $rc || exit $rc
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline --no-host-path > $O/bench_under_rocprof.json 2> $O/kt.err; rc=$?
  echo "kt rc=$rc"
)
}

# round 4: host leg last (default) vs first in the full bench line (placement / THP A/B)
gpu_r4_hostorder() {
(
  for order in last first; do
    extra="--host-path-last"; [ $order = first ] && extra=""
    timeout -k 10 400 python3 bench.py --steps 50 --no-cpu-baseline $extra > gpurun_out/r4_hostorder_$order.json 2>> gpurun_out/r4_hostorder.err; rc=$?
    echo "$order rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_hostorder_$order.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m]['numa_node_rank0'], d[m]['cpu_core_s_per_step_rank0'], d[m].get('copy_ms_per_step_rank0'), d[m].get('wait_ms_per_step_rank0')) for m in d})")"
    ok_rc $rc || exit $rc
  done
  grep -i AnonHugePages /proc/meminfo; cat /sys/kernel/mm/transparent_hugepage/enabled; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6; cat /proc/self/cgroup
)
}

# round 4: the pageable pipeline's depth — host leg last in the full bench line, chunk MiB x slots
gpu_r4_slots() {
(
  timeout -k 10 300 python -u -m pytest tests/test_gpu_hostpath.py tests/test_gpu_ptrs.py -q --timeout 120 --timeout-method thread > gpurun_out/r4_slots_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -1 gpurun_out/r4_slots_tests.log; ok_rc $rc || exit $rc
  for cfg in "16 2" "16 4" "64 2" "64 4" "32 4"; do
    set -- $cfg
    TCPCSUM_HOST_CHUNK_MB=$1 TCPCSUM_HOST_SLOTS=$2 timeout -k 10 400 python3 bench.py --steps 50 --no-cpu-baseline > gpurun_out/r4_slots_$1_$2.json 2>> gpurun_out/r4_slots.err; rc=$?
    echo "chunk=$1 slots=$2 rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_slots_$1_$2.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m]['numa_node_rank0'], d[m].get('copy_ms_per_step_rank0'), d[m].get('wait_ms_per_step_rank0')) for m in d})")"
    ok_rc $rc || exit $rc
  done
)
}

# round 4: host leg last in the full line, its context created late (control) or at the start
# of the run (--host-ctx-early), and the leg run first — does allocation order explain the
# pageable slowdown?
gpu_r4_early() {
(
  for v in late early first late2 early2; do
    case $v in late*) extra="--host-path-last";; early*) extra="--host-path-last --host-ctx-early";; first) extra="";; esac
    timeout -k 10 400 python3 bench.py --steps 50 --no-cpu-baseline $extra > gpurun_out/r4_early_$v.json 2>> gpurun_out/r4_early.err; rc=$?
    echo "$v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_early_$v.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m]['numa_node_rank0'], d[m].get('copy_ms_per_step_rank0'), d[m].get('wait_ms_per_step_rank0')) for m in d})")"
    ok_rc $rc || exit $rc
  done
)
}

# round 4: which device leg leaves the pageable host pipeline slow — the headline alone with
# many or few steps, host leg last
gpu_r4_culprit() {
(
  for v in "h50:--steps 50" "h2:--steps 2 --warmup 1" "probe2:--steps 2 --warmup 1 --probe" "all2:--steps 2 --warmup 1 --other"; do
    name=${v%%:*}; a=${v#*:}
    case $a in *--other) a=${a% --other}; oc="";; *--probe) a=${a% --probe}; oc="--no-other-configs";; *) oc="--no-other-configs --no-probe";; esac
    timeout -k 10 400 python3 bench.py --no-cpu-baseline --host-path-last $a $oc > gpurun_out/r4_culprit_$name.json 2>> gpurun_out/r4_culprit.err; rc=$?
    echo "$name rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_culprit_$name.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m].get('copy_ms_per_step_rank0'), d[m].get('wait_ms_per_step_rank0')) for m in d})")"
    ok_rc $rc || exit $rc
  done
)
}

gpu_r4_bisect() {
(
  for o in 64k 64 wire; do
    timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --no-probe --host-path-last --other $o > gpurun_out/r4_bisect_$o.json 2>> gpurun_out/r4_bisect.err; rc=$?
    echo "$o rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_bisect_$o.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m].get('copy_ms_per_step_rank0'), d[m].get('wait_ms_per_step_rank0')) for m in d})")"
    ok_rc $rc || exit $rc
  done
)
}

# round 4: after the 64k batch, which part of the pageable pipeline is slow — DMA to HBM or the
# kernel reading staging over PCIe; 4 slots; HIP's own event waits spinning or yielding
gpu_r4_dma() {
(
  for v in "dflt:" "nodma:TCPCSUM_HOST_DMA=0" "slots4:TCPCSUM_HOST_SLOTS=4" "nocache:PYTORCH_NO_HIP_MEMORY_CACHING=1"; do
    name=${v%%:*}; e=${v#*:}
    env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --no-probe --host-path-last --other 64k > gpurun_out/r4_dma_$name.json 2>> gpurun_out/r4_dma.err; rc=$?
    echo "$name rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_dma_$name.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m].get('copy_ms_per_step_rank0'), d[m].get('wait_ms_per_step_rank0'), d[m].get('raw_pinned_h2d_GiB/s')) for m in d})")"
    ok_rc $rc || exit $rc
  done
)
}

# round 4: the uniform host paths on one stream (64 MiB staging, 256 MiB DMA pieces) — every
# GPU test, then the host leg first (default), last after the 64k batch, and last after all
gpu_r4_onestream() {
(
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${R4OS:-r4_onestream}_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/${R4OS:-r4_onestream}_tests.log | tail -1; grep FAILED gpurun_out/${R4OS:-r4_onestream}_tests.log | head; ok_rc $rc || exit $rc
  for v in "first:--steps 50" "last64k:--steps 2 --warmup 1 --no-probe --host-path-last --other 64k" "lastall:--steps 50 --host-path-last"; do
    name=${v%%:*}; a=${v#*:}
    timeout -k 10 400 python3 bench.py --no-cpu-baseline $a > gpurun_out/${R4OS:-r4_onestream}_$name.json 2>> gpurun_out/r4_onestream.err; rc=$?
    echo "$name rc=$rc $(python3 -c "import json; D=json.load(open('gpurun_out/${R4OS:-r4_onestream}_$name.json')); d=D['host_path']; print(D['value'], {m: (d[m]['GiB/s'], d[m].get('copy_ms_per_step_rank0'), d[m].get('wait_ms_per_step_rank0'), d[m].get('raw_pinned_h2d_GiB/s'), d[m]['cpu_core_s_per_step_rank0']) for m in d})")"
    ok_rc $rc || exit $rc
  done
)
}

# round 4: DMA piece size for page-locked uniform batches (HBM the context holds), and the
# pageable chunk cap, interleaved twice — host leg only
gpu_r4_pieces() {
(
  for rep in 1 2; do
    for cfg in "256 128" "1024 128" "512 256"; do
      set -- $cfg
      TCPCSUM_HOST_DMA_CHUNK_MB=$1 TCPCSUM_HOST_CHUNK_MB=$2 timeout -k 10 200 python3 bench.py --host-path-only --host-steps 10 > gpurun_out/r4_pieces_$1_$2_rep$rep.json 2>> gpurun_out/r4_pieces.err; rc=$?
      echo "dma=$1 chunk=$2 rep=$rep rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_pieces_$1_$2_rep$rep.json'))['host_path']; print({m: (d[m]['GiB/s'], d[m].get('raw_pinned_h2d_GiB/s'), d[m]['cpu_core_s_per_step_rank0']) for m in d})")"
      ok_rc $rc || exit $rc
    done
  done
)
}

# round 4, last: the final rehearsal at HEAD plus the seam's default and pinned-pool latency /
# core-us beside the reference's one-core checksum
gpu_r4_final2() {
(
  gpu_r4_final || exit $?
  O=gpurun_out/r4final
  for v in "cpu:cpu:" "staged:gpu:" "pinned:gpu:pinned"; do
    IFS=: read name mode extra <<< "$v"
    if [ $mode = gpu ]; then
      env -u TCPCSUM_PRELOAD_TX LD_PRELOAD=$PWD/tcp_amd/libtcpcsum_preload.so TCPCSUM_PRELOAD_ANY_SOCKET=1 TCPCSUM_PRELOAD_TX=fill \
        timeout -k 10 120 tools/mmsg_bench gpu 300 $extra > $O/seam_$name.json 2> $O/seam_$name.err; rc=$?
    else
      timeout -k 10 120 tools/mmsg_bench cpu 300 > $O/seam_$name.json 2> $O/seam_$name.err; rc=$?
    fi
    echo "seam $name rc=$rc $(cat $O/seam_$name.json)"; ok_rc $rc || exit $rc
  done
)
}

# round 4: staging-slot waits sleeping (default with the blocking wait) vs spinning, host leg
# only, interleaved four times
gpu_r4_slotwait() {
(
  for rep in 1 2 3 4; do
    for sl in 1 0; do
      TCPCSUM_HOST_SLOT_SLEEP=$sl timeout -k 10 200 python3 bench.py --host-path-only --host-steps 10 > gpurun_out/r4_slotwait_s${sl}_rep$rep.json 2>> gpurun_out/r4_slotwait.err; rc=$?
      echo "sleep=$sl rep=$rep rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_slotwait_s${sl}_rep$rep.json'))['host_path']['pageable']; print(d['GiB/s'], d['cpu_core_s_per_step_rank0'], d['copy_ms_per_step_rank0'], d['wait_ms_per_step_rank0'])")"
      ok_rc $rc || exit $rc
    done
  done
)
}

# round 4: how many threads the pageable uniform path copies on (the DMA, not the copy, is
# the bound), host leg only, interleaved twice
gpu_r4_bulk() {
(
  for rep in 1 2; do
    for t in 2 3 4 0; do
      TCPCSUM_HOST_BULK_THREADS=$t timeout -k 10 200 python3 bench.py --host-path-only --host-steps 10 > gpurun_out/r4_bulk_t${t}_rep$rep.json 2>> gpurun_out/r4_bulk.err; rc=$?
      echo "threads=$t rep=$rep rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_bulk_t${t}_rep$rep.json'))['host_path']['pageable']; print(d['GiB/s'], d['cpu_core_s_per_step_rank0'], d['copy_ms_per_step_rank0'], d['wait_ms_per_step_rank0'], d['copy_threads'])")"
      ok_rc $rc || exit $rc
    done
  done
)
}

# round 4: staged wire batches through the sendmmsg seam with plain memcpy (default) vs
# streaming stores from 64-B starts (TCPCSUM_HOST_WIRE_NT=1), interleaved four times; the
# seam tests with the streaming variant first
gpu_r4_wirent() {
(
  TCPCSUM_HOST_WIRE_NT=1 timeout -k 10 300 python -u -m pytest tests/test_seam.py tests/test_gpu_ptrs.py tests/test_plumbing.py -q --timeout 120 --timeout-method thread > gpurun_out/r4_wirent_tests.log 2>&1; rc=$?
  echo "tests(nt) rc=$rc"; grep -E "passed|failed" gpurun_out/r4_wirent_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
  for rep in 1 2 3 4; do
    for nt in 0 1; do
      env LD_PRELOAD=$PWD/tcp_amd/libtcpcsum_preload.so TCPCSUM_PRELOAD_ANY_SOCKET=1 TCPCSUM_PRELOAD_TX=fill TCPCSUM_HOST_WIRE_NT=$nt \
        timeout -k 10 120 tools/mmsg_bench gpu 300 > gpurun_out/r4_wirent_nt${nt}_rep$rep.json 2>> gpurun_out/r4_wirent.err; rc=$?
      echo "nt=$nt rep=$rep rc=$rc $(cat gpurun_out/r4_wirent_nt${nt}_rep$rep.json)"; [ $rc -eq 0 ] || exit $rc
    done
  done
)
}

# round 4: the pageable copy's escalation to every copy thread once the copy, not the DMA, is
# the bound — default (4 threads) vs forced 1 and 2 threads, host leg only
gpu_r4_escal() {
(
  timeout -k 10 300 python -u -m pytest tests/test_gpu_hostpath.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/r4_escal_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_escal_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
  for v in dflt1:4 bulk1:1 dflt2:4 bulk2:2; do
    n=${v%%:*}; t=${v#*:}
    TCPCSUM_HOST_BULK_THREADS=$t timeout -k 10 200 python3 bench.py --host-path-only --host-steps 10 > gpurun_out/r4_escal_$n.json 2>> gpurun_out/r4_escal.err; rc=$?
    echo "$n threads=$t rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r4_escal_$n.json'))['host_path']['pageable']; print(d['GiB/s'], d['cpu_core_s_per_step_rank0'], d['copy_ms_per_step_rank0'], d['wait_ms_per_step_rank0'])")"
    ok_rc $rc || exit $rc
  done
)
}

# round 4: the recvmmsg side — 1024 packets over UDP loopback, one recvmmsg timed: plain, under
# the interposer (RX=drop: GPU verify), and plain + CPU verify per packet; twice
gpu_r4_rx() {
(
  for rep in 1 2; do
    timeout -k 10 120 tools/mmsg_bench rx 300 > gpurun_out/r4_rx_plain_$rep.json 2>> gpurun_out/r4_rx.err || exit $?
    env LD_PRELOAD=$PWD/tcp_amd/libtcpcsum_preload.so TCPCSUM_PRELOAD_ANY_SOCKET=1 TCPCSUM_PRELOAD_TX=off TCPCSUM_PRELOAD_RX=drop \
      timeout -k 10 120 tools/mmsg_bench rx 300 > gpurun_out/r4_rx_gpu_$rep.json 2>> gpurun_out/r4_rx.err || exit $?
    timeout -k 10 120 tools/mmsg_bench rxcpu 300 > gpurun_out/r4_rx_cpu_$rep.json 2>> gpurun_out/r4_rx.err || exit $?
    for v in plain gpu cpu; do echo "$v rep=$rep $(cat gpurun_out/r4_rx_${v}_$rep.json)"; done
  done
)
}

# round 3: wire FILL line store (default) — every GPU test first, then the A/B timing three
# times (the two FILL stores must agree byte for byte every time)
gpu_r3_fill() {
(
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gputest_fill_line.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gputest_fill_line.log
  if [ $rc -eq 0 ]; then
    for i in 1 2 3; do
      timeout -k 10 200 python tools/fill_line_ab.py --rounds 2 >> gpurun_out/fill_line_ab2.jsonl 2> gpurun_out/fill_line_ab.err || { echo "ab failed"; exit 1; }
    done
    echo ab ok
  fi
)
}

# round 3: the wire FILL change under every GPU test and the A/B, then an N=8 rehearsal of
# bench.py on one GPU (all eight ranks share it; every rank checks its 8Mx1500 shard digest)
gpu_r3_n8() {
(
  gpu_r3_fill || exit 1
  TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 8 --steps 5 --warmup 2 --no-other-configs > gpurun_out/bench_n8_shared.json 2> gpurun_out/bench_n8_shared.err
  echo "n8 rc=$?"; cat gpurun_out/bench_n8_shared.json | cut -c1-400
)
}

# gpu_round3
gpu_round3() {
(
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gputest_r3b.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/gputest_r3b.log | grep -E "passed|failed|FAILED|Error" 
  if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 6 > gpurun_out/bench_r3b.json 2> gpurun_out/bench_r3b.err; echo "bench rc=$?"
  fi
)
}

# New uniform default (blocks 0) against the previous caps (512 / 4096) at small and MTU sizes.
grid_check() {
(
  set -e
  O=gpurun_out/grid_check
  mkdir -p $O
  for L in 64 100 128 200 256 576 1024 1500; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,512,4096 --unrolls 0 --rounds 5 --steps 20 > $O/len$L.jsonl 2>>$O/err
  done
)
}

# One-wave-per-segment uniform batches (shape 9): default grid against larger ones.
grid_long() {
(
  set -e
  O=gpurun_out/grid_long
  mkdir -p $O
  for L in 9000 12300 20004 65536; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,4096,16384,16777216 --unrolls 0 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
  done
)
}

# Byte-granular (M1) uniform batches: the 4096-workgroup default against larger grids.
grid_m1() {
(
  set -e
  O=gpurun_out/grid_m1
  mkdir -p $O
  for L in 99 577 1499 3001; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,16384,65536,16777216 --unrolls 0,2 --rounds 5 --steps 20 > $O/len$L.jsonl 2>>$O/err
  done
)
}

# Default grid vs one tile per wave (max_blocks uncapped) for the uniform kernel
# across the bench configs and a few mid sizes (tools/sweep.py, interleaved rounds).
grid_sweep() {
(
  set -e
  O=gpurun_out/grid_sweep
  mkdir -p $O
  timeout -k 10 200 python3 tools/sweep.py --config 64 --blocks 0,4096,16384,65536,262144 --unrolls 0 --rounds 5 --steps 30 > $O/c64.jsonl 2>>$O/err
  timeout -k 10 200 python3 tools/sweep.py --config 64k --blocks 0,1024,4096,65536 --unrolls 0 --rounds 5 --steps 10 > $O/c64k.jsonl 2>>$O/err
  for L in 256 576 4096 8192; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,16384,65536,262144 --unrolls 0 --rounds 5 --steps 20 > $O/len$L.jsonl 2>>$O/err
  done
  timeout -k 10 200 python3 tools/sweep.py --config 1500 --blocks 0,16384 --unrolls 0 --rounds 7 --steps 30 --probe > $O/c1500.jsonl 2>>$O/err
)
}

# 64 KiB config: why bench.py (2.47 ms) and the sweep (2.40 ms) differ — steps, warmup, shape.
k64_check() {
(
  set -e
  O=gpurun_out/k64
  mkdir -p $O
  B="python3 bench.py --config 64k --no-cpu-baseline --no-other-configs"
  for s in 5 40; do
    timeout -k 10 120 $B --steps $s --warmup 3 > $O/bench_s$s.json 2>>$O/err
    timeout -k 10 120 $B --steps $s --warmup 3 --shape 9 > $O/bench_s${s}_shape9.json 2>>$O/err
  done
  timeout -k 10 200 python3 tools/sweep.py --config 64k --shapes 9,13 --blocks 0 --unrolls 0 --rounds 2 --steps 40 > $O/sweep_s40.jsonl 2>>$O/err
)
}

# Balanced kernels: per-lane sums for tiles of small segments, against the previous build.
lane_ab() {
(
  set -e
  O=gpurun_out/lane
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
  timeout -k 10 300 python3 tools/lb_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/lb_ab.jsonl 2> $O/lb_ab.err
)
}

# lb_sweep
lb_sweep() {
(
  set -e
  for cfg in "0,0,9,0 0,0,8,0" "1024,0,8,0 1024,0,7,0" "2048,0,8,0 2048,0,7,0" "16384,0,8,0 16384,0,7,0"; do
    set -- $cfg
    LB_HEAD_WIRE=$1 LB_HEAD_DESC=$2 timeout -k 10 120 python3 tools/lb_ab.py tcp_amd/ab/libtcpcsum_r02a.so > gpurun_out/lbsweep_$1.jsonl 2>>gpurun_out/lbsweep.err
  done
)
}

# Wire shape 10 (window chunks through LDS) against the lane-group defaults.
lds_ab() {
(
  set -e
  O=gpurun_out/lds
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread -k "ipv4 or fuzz or ptrs" > $O/parity.log 2>&1
  for S in 1536 1024 2048; do
    SLOT=$S SHAPES=-1,5,7,10 BLOCKS=0 UNROLLS=1 timeout -k 10 300 python3 tools/wiresweep.py > $O/slot$S.jsonl 2>> $O/err
  done
)
}

# pmc_64
pmc_64() {
(
  set -e
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  B="python3 bench.py --steps 60 --warmup 5 --no-other-configs --no-cpu-baseline --probe"
  for cfg in 64 64k; do
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_fetch -o p -- $B --config $cfg > gpurun_out/pmc_${cfg}_fetch.log 2>&1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_write -o p -- $B --config $cfg > gpurun_out/pmc_${cfg}_write.log 2>&1
  done
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_64 -o p -- $B --config 64 > gpurun_out/kt_64.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_64_sq -o p -- $B --config 64 > gpurun_out/pmc_64_sq.log 2>&1
)
}

# Counters for the balanced wire kernel on packed IMIX only (tools/lb_ab.py workload).
pmc_imix() {
(
  set -e
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  O=gpurun_out/pmc_imix
  mkdir -p $O
  export LB_ONLY=ipv4_lb_1M_imix_packed_verify
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/a -o p -- python3 tools/lb_ab.py > $O/a.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- python3 tools/lb_ab.py > $O/b.log 2>&1
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 tools/lb_ab.py > $O/kt.log 2>&1
  echo done
)
}

# Counters for the balanced wire kernel on packed IMIX (tools/lb_ab.py workloads), one pass each.
pmc_lb() {
(
  set -e
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  O=gpurun_out/pmc_lb
  mkdir -p $O
  timeout -k 10 120 ./tests/c/abi_smoke --gpu > $O/abi_smoke.log 2>&1
  P="python3 tools/lb_ab.py"
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/a -o p -- $P > $O/a.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- $P > $O/b.log 2>&1
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $P > $O/kt.log 2>&1
  echo done
)
}

# Round-3 evidence on one MI355X (through gpurun): rocprofv3 kernel trace of the
# headline bench (its average must agree with bench.py's HIP events), FETCH_SIZE
# of the headline kernel, FETCH/WRITE_SIZE of the 64-B multi-batch launch, and
# WRITE_SIZE / FETCH_SIZE of the wire FILL stores (2-byte vs line vs VERIFY).
# Every pass is its own run (rocprofv3 does not split counters over passes).
round3_profile() {
(
  O=gpurun_out/r3prof
  mkdir -p $O
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  B="python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline --probe"
  run() { echo "== $1"; shift; "$@" || { echo "failed: $?"; exit 1; }; }
  run kt timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $B > $O/bench_under_rocprof.json 2> $O/kt.err
  run fetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- $B > $O/pmc_fetch.log 2>&1
  M="python3 tools/multi_sweep.py --ks 16 --unrolls 4 --grids 0 --rounds 1 --steps 10"
  run mfetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_multi_fetch -o p -- $M > $O/pmc_multi_fetch.log 2>&1
  run mwrite timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_multi_write -o p -- $M > $O/pmc_multi_write.log 2>&1
  W="python3 tools/wire_fill_pmc.py"
  run wwrite timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_wire_write -o p -- $W > $O/pmc_wire_write.log 2>&1
  run wfetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_wire_fetch -o p -- $W > $O/pmc_wire_fetch.log 2>&1
  run wkt timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_wire -o k -- $W > $O/kt_wire.log 2>&1
  echo done
)
}

# Round-4 evidence: rocprofv3 kernel trace of the headline bench, FETCH_SIZE of the headline
# kernel (traffic.json "1500"), WRITE_SIZE / FETCH_SIZE / kernel trace of the wire FILL stores
# (the FILL instantiation no longer spills: its scratch write-back should be gone).
round4_profile() {
(
  O=gpurun_out/r4prof
  mkdir -p $O
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  B="python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline --no-host-path"
  run() { echo "== $1"; shift; "$@" || { echo "failed: $?"; exit 1; }; }
  run kt timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $B > $O/bench_under_rocprof.json 2> $O/kt.err
  run fetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- $B > $O/pmc_fetch.log 2>&1
  W="python3 tools/wire_fill_pmc.py"
  run wwrite timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_wire_write -o p -- $W > $O/pmc_wire_write.log 2>&1
  run wfetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_wire_fetch -o p -- $W > $O/pmc_wire_fetch.log 2>&1
  run wkt timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_wire -o k -- $W > $O/kt_wire.log 2>&1
  echo done
)
}

# Round-end evidence (gpurun): GPU tests, smoke, default bench, N=2 rehearsal on one GPU
# (TCPCSUM_BENCH_SHARE_DEVICE=1: both ranks on cuda:0), rocprofv3 kernel trace of the headline.
round_final() {
(
  set -e
  O=gpurun_out/final
  mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
  TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 50 > $O/bench_n2_shared.json 2> $O/bench_n2.err
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/kt.err
  echo done
)
}

# Round-end evidence on one MI355X (run through gpurun): GPU tests, smoke, the
# default bench line, and rocprofv3 summaries of the headline kernel — kernel
# trace (average duration must agree with bench.py's HIP events) and a separate
# FETCH_SIZE pass (traffic) — plus WRITE_SIZE of the wire FILL. Outputs under
# gpurun_out/round/; copy what is judged into profiles/.
round_profile() {
(
  set -e
  R=${1:-r02}
  O=gpurun_out/round
  mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  B="python3 bench.py --steps 100 --no-other-configs --no-cpu-baseline --probe"
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $B > $O/bench_under_rocprof.json 2> $O/kt.err
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- $B > $O/pmc_fetch.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_wire_write -o p -- python3 tools/fillbench.py > $O/pmc_wire_write.log 2>&1
  echo done
)
}

# Split-segment kernel (shape 13: four waves per segment) against the
# one-wave-per-segment kernel (shape 9) on long uniform segments.
split_sweep() {
(
  set -e
  O=gpurun_out/split
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "forced_shapes or long_segments or two_fold or all_unrolls" > $O/parity.log 2>&1
  for L in 12300 20004 32768 65536 131072; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --shapes 9,13 --blocks 0 --unrolls 0,2,4,8 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
  done
  timeout -k 10 300 python3 tools/sweep.py --config 64k --shapes 9,13 --blocks 0 --unrolls 0,2,4,8 --rounds 3 --steps 5 > $O/cfg64k.jsonl 2>>$O/err
)
}

# Split-segment kernel (shape 13) vs shape 9, second pass: jumbo / byte-granular / aligned mid sizes.
split_sweep2() {
(
  set -e
  O=gpurun_out/split2
  mkdir -p $O
  for L in 9000 8999 12301 16384 24576 49152 65536 65532; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --shapes 9,13 --blocks 0 --unrolls 0,1,2 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
  done
  timeout -k 10 300 python3 tools/sweep.py --config 64k --shapes 9,13 --blocks 0,1024,4096 --unrolls 0,2 --rounds 3 --steps 5 > $O/cfg64k.jsonl 2>>$O/err
)
}

# Balanced ragged kernel with segments-per-wave sized by max_len: parity, sweep, A/B vs the previous build.
spw_check() {
(
  set -e
  O=gpurun_out/spw
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -k "desc or balanced or fuzz" > $O/parity.log 2>&1
  SIZES=1500,4096,9000,32768,65536 SHAPES=-1,4,5,6,8 ROUNDS=3 timeout -k 10 400 python3 tools/desc_sweep.py > $O/desc.jsonl 2> $O/err
  timeout -k 10 300 python3 tools/lb_ab.py tcp_amd/ab/libtcpcsum_prev.so > $O/lb_ab.jsonl 2>> $O/err
)
}

# Segment builder shapes across payload sizes (pure ACK .. jumbo).
tx_size_sweep() {
(
  set -e
  O=gpurun_out/txs
  mkdir -p $O
  for L in 0 40 536 1456 4000 8956; do
    TX_LEN=$L TX_SHAPES=-1,0,1,2,3,4 TX_BLOCKS=32768 TX_UNROLLS=1 timeout -k 10 300 python3 tools/txbench.py --sweep > $O/len$L.jsonl 2>> $O/err
  done
)
}

# Segment builder: (16,2) vs (32,3) lane groups between 256 B and 1.2 KiB payloads.
tx_size_sweep2() {
(
  set -e
  O=gpurun_out/txs2
  mkdir -p $O
  for L in 256 536 768 1024 1200; do
    TX_LEN=$L TX_SHAPES=2,1,2,1 TX_BLOCKS=32768 TX_UNROLLS=1 timeout -k 10 300 python3 tools/txbench.py --sweep > $O/len$L.jsonl 2>> $O/err
  done
)
}

# Uniform batches across sizes: the auto plan against every shape that covers the size.
uniform_size_sweep() {
(
  set -e
  O=gpurun_out/usz
  mkdir -p $O
  for L in 40 200 576 1024 2048 3000 4096 6000 8192; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --shapes=-1,2,3,4,5,6,7,8,9,12,13 --blocks 0 --unrolls 0 --rounds 3 --steps 10 > $O/len$L.jsonl 2>>$O/err
  done
)
}

# Uniform 6-8 KiB segments: shape 8 (64 lanes x 8 chunks) against one wave (9) and four waves (13) per segment.
uniform_size_sweep2() {
(
  set -e
  O=gpurun_out/usz2
  mkdir -p $O
  for L in 6400 7000 7600 8000 8192; do
    timeout -k 10 200 python3 tools/sweep.py --len $L --shapes=-1,9,13 --blocks 0 --unrolls 0,1 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
  done
)
}

# Wire lane-group shapes on packets between the MTU and jumbo sizes (slots 2-9 KiB).
wire_big_sweep() {
(
  set -e
  O=gpurun_out/wbig
  mkdir -p $O
  for S in 2048 3072 4608 9216; do
    SLOT=$S SHAPES=-1,1,2,4,7 BLOCKS=0 UNROLLS=1,2 timeout -k 10 300 python3 tools/wiresweep.py > $O/slot$S.jsonl 2>> $O/err
  done
)
}

# Wire defaults after the size-class rule: parity, then the default shape per slot size.
wire_default_check() {
(
  set -e
  O=gpurun_out/wdef
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread -k "ipv4 or fuzz or ptrs" > $O/parity.log 2>&1
  for S in 1536 2048 3072 4608 9216; do
    SLOT=$S SHAPES=-1,1,7 BLOCKS=0 UNROLLS=1 timeout -k 10 300 python3 tools/wiresweep.py > $O/slot$S.jsonl 2>> $O/err
  done
)
}

# Balanced wire kernel on 64K-128K-packet batches: auto (>= 4096 wave tiles) vs forced 64-packet tiles.
wire_lb_small() {
(
  set -e
  O=gpurun_out/wlbs
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_ptrs.py -x -q --timeout 120 --timeout-method thread -k "ipv4 or fuzz or ptrs" > $O/parity.log 2>&1
  for N in 65536 131072; do
    N=$N SLOT=84 PAYLOAD=40 SHAPES=-1,8,0 BLOCKS=0 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py > $O/s84_n$N.jsonl 2>> $O/err
    N=$N SLOT=576 PAYLOAD=496 SHAPES=-1,8,7 BLOCKS=0 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py > $O/s576_n$N.jsonl 2>> $O/err
  done
)
}

# wire_mid_sweep
wire_mid_sweep() {
(
  set -e
  for sp in "768 688" "896 816"; do
    set -- $sp
    SLOT=$1 PAYLOAD=$2 SHAPES=8,7 BLOCKS=0,16384 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py | grep -v round > gpurun_out/wire_mtu_sweep_$1.jsonl
  done
)
}

# Lane-group wire kernel shapes across slot sizes, VERIFY and FILL (tools/wiresweep.py):
# auto (-1), 5 (8 x 12 chunks), 7 (8 x 4 chunks, more rounds), 8 (balanced).
wire_mtu_sweep() {
(
  set -e
  for sp in "576 496" "1024 944" "1536 1456"; do
    set -- $sp
    SLOT=$1 PAYLOAD=$2 SHAPES=${SHAPES:--1,5,7,8} BLOCKS=${BLOCKS:-0,16384} UNROLLS=1 timeout -k 10 200 \
      python3 tools/wiresweep.py | grep -v round > gpurun_out/wire_mtu_sweep_$1.jsonl
  done
)
}

# Wire shapes on small device-resident batches of MTU packets (1536-B slots).
wire_small_sweep() {
(
  set -e
  O=gpurun_out/wsm
  mkdir -p $O
  for N in 1024 8192 32768; do
    N=$N SHAPES=-1,1,3,5,7 BLOCKS=0 UNROLLS=1 timeout -k 10 200 python3 tools/wiresweep.py > $O/n$N.jsonl 2>> $O/err
  done
)
}

# Host-path check after a host-code change: its GPU tests, the staged/in-place
# sweep and the end-to-end rates (gpurun_out/hp/)
hostpath_check() {
(
  O=gpurun_out/hp
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ptrs.py tests/test_plumbing.py tests/test_seam.py tests/test_gpu_hostpath.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
  tail -1 $O/t.log
  timeout -k 10 400 python3 tools/hostpath_sweep.py --rounds 3 > $O/sweep.jsonl 2> $O/sweep.err || { tail $O/sweep.err; exit 1; }
  timeout -k 10 200 python3 tools/e2e.py > $O/e2e.jsonl 2> $O/e2e.err || { tail $O/e2e.err; exit 1; }
  echo hostpath ok
)
}

# Round 3 rehearsal of the driver's round-end steps at HEAD: every GPU test, smoke(), the
# default bench line (the driver's command), then the host-path end-to-end rates.
round3_final() {
(
  O=gpurun_out/final3
  mkdir -p $O
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -5 $O/gputest.log; exit 1; }
  tail -1 $O/gputest.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  timeout -k 10 300 python3 tools/e2e.py > $O/e2e.jsonl 2> $O/e2e.err || { tail $O/e2e.err; exit 1; }
  echo final ok
)
}

# The segment builder against the chip's read+write ceiling: tools/copy_probe (plain 16-B
# copies of the builder's 1.53 GB of payload, store policies, 44-B destination shift) and
# tools/txbench.py (k_tx_build, and torch copy_ as before) in the same box.
copy_ceiling() {
(
  O=gpurun_out/copy
  mkdir -p $O
  timeout -k 10 200 ./tools/copy_probe > $O/copy_probe.jsonl 2> $O/copy_probe.err || { tail $O/copy_probe.err; exit 1; }
  timeout -k 10 200 python3 tools/txbench.py > $O/txbench.jsonl 2> $O/txbench.err || { tail $O/txbench.err; exit 1; }
  echo copy ok
)
}

# Segment builder launch shapes up to one tile per wave (1M x 1456-B payloads)
tx_grid_sweep() {
(
  O=gpurun_out/txgrid
  mkdir -p $O
  TX_SHAPES=2,3,4 TX_BLOCKS=16384,32768,65536,131072,262144 TX_UNROLLS=1,2 timeout -k 10 300 python3 tools/txbench.py --sweep > $O/sweep.jsonl 2> $O/sweep.err || { tail $O/sweep.err; exit 1; }
  echo txgrid ok
)
}

# Segment builder A/B against the builds in tcp_amd/ab/ (tools/tx_ab.py --build, on the CPU first)
tx_ab() {
(
  O=gpurun_out/txab
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "tx_build" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -15 $O/t.log; exit 1; }
  tail -1 $O/t.log
  timeout -k 10 300 python3 tools/tx_ab.py > $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  cat $O/ab.jsonl
)
}

# Segment builder after a kernel change: its parity tests, txbench (store policies), and a
# launch-shape sweep of the default shape
tx_check() {
(
  O=gpurun_out/txcheck
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "tx_build" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -15 $O/t.log; exit 1; }
  tail -1 $O/t.log
  timeout -k 10 200 python3 tools/txbench.py > $O/txbench.jsonl 2> $O/txbench.err || { tail $O/txbench.err; exit 1; }
  TX_SHAPES=${TX_SHAPES:-2} TX_BLOCKS=${TX_BLOCKS:-16384,32768,65536,131072} TX_UNROLLS=${TX_UNROLLS:-1,2} timeout -k 10 300 python3 tools/txbench.py --sweep > $O/sweep.jsonl 2> $O/sweep.err || { tail $O/sweep.err; exit 1; }
  grep -v sweep $O/txbench.jsonl
)
}

# Builder shapes by payload size, interleaved (tools/txbench.py --sweep per TX_LEN)
tx_size_ab() {
(
  O=gpurun_out/txsize
  mkdir -p $O
  for L in ${TX_LENS:-256 536 1024 1200 1456 4000 9000}; do
    TX_LEN=$L TX_SHAPES=${TX_SHAPES:-1,2,4,5,1,2,4,5} TX_BLOCKS=32768 TX_UNROLLS=1 timeout -k 10 200 python3 tools/txbench.py --sweep > $O/len$L.jsonl 2> $O/err || { tail $O/err; exit 1; }
  done
  echo txsize ok
)
}

# Wire kernel A/B against tcp_amd/ab/libtcpcsum_wire*.so, after its GPU tests
wire_ab() {
(
  O=gpurun_out/wireab
  mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_plumbing.py tests/test_gpu_ptrs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -15 $O/t.log; exit 1; }
  tail -1 $O/t.log
  timeout -k 10 400 python3 tools/wire_lib_ab.py > $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  cat $O/ab.jsonl
)
}

# Copy threads on the GPU's NUMA node or anywhere: host-path tests, sweep (numa 0/1), e2e
numa_check() {
(
  O=gpurun_out/numa
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ptrs.py tests/test_plumbing.py tests/test_seam.py tests/test_gpu_hostpath.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -15 $O/t.log; exit 1; }
  tail -1 $O/t.log
  timeout -k 10 400 python3 tools/hostpath_sweep.py --rounds 3 > $O/sweep.jsonl 2> $O/sweep.err || { tail $O/sweep.err; exit 1; }
  TCPCSUM_HOST_NUMA=0 timeout -k 10 200 python3 tools/e2e.py > $O/e2e_numa0.jsonl 2> $O/e2e0.err || { tail $O/e2e0.err; exit 1; }
  timeout -k 10 200 python3 tools/e2e.py > $O/e2e_numa1.jsonl 2> $O/e2e1.err || { tail $O/e2e1.err; exit 1; }
  echo numa ok
)
}

if [ $# -eq 0 ]; then
  echo "experiments: numa_check wire_ab tx_size_ab tx_check tx_ab tx_grid_sweep copy_ceiling round3_final hostpath_check gpu_r3_fill gpu_r3_n8 gpu_round3 grid_check grid_long grid_m1 grid_sweep k64_check lane_ab lb_sweep lds_ab pmc_64 pmc_imix pmc_lb round3_profile round_final round_profile split_sweep split_sweep2 spw_check tx_size_sweep tx_size_sweep2 uniform_size_sweep uniform_size_sweep2 wire_big_sweep wire_default_check wire_lb_small wire_mid_sweep wire_mtu_sweep wire_small_sweep"
  exit 0
fi
"$@"
