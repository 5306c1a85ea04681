#!/usr/bin/env bash
# Round-5 GPU runs (one function per experiment; outputs under gpurun_out/r5/):
#   bash tools/r5_runs.sh <function> [args]
# Every GPU step runs under its own timeout and the steps are chained: the first
# failure ends the call.
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
PRE=$PWD/tcp_amd/libtcpcsum_preload.so

ok_rc() { [ "$1" = 0 ]; }

# GPU tests of the files named (default: all), one pytest process
tests() {
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "${@:-tests}" \
    > $O/gputest.txt 2>&1; rc=$?
  tail -5 $O/gputest.txt; return $rc
}

# the sendmmsg / recvmmsg seam per 1024 x 1500-B batch: reference CPU checksum; staged (loop.c's
# malloc'd buffers); TCPCSUM_PRELOAD_POOL=mmsg_bench (the same mallocs served from the interposer's
# page-locked arena, loop.c unedited); level 2 (out-buffers carved from tcpcsum_host_alloc by the
# application). rx: plain recvmmsg, rx drop staged / pool, CPU verify. Interleaved, $1 rounds.
seam() {
  local reps=${1:-3}
  for rep in $(seq 1 $reps); do
    for v in "cpu:cpu::" "staged:gpu::" "pool:gpu::mmsg_bench" "pinned:gpu:pinned:"; do
      IFS=: read name mode extra pool <<< "$v"
      if [ $mode = gpu ]; then
        # LD_PRELOAD on the measured program only (env execs it), never on timeout
        timeout -k 10 120 env LD_PRELOAD=$PRE TCPCSUM_PRELOAD_ANY_SOCKET=1 TCPCSUM_PRELOAD_TX=fill \
          TCPCSUM_PRELOAD_STATS=1 TCPCSUM_PRELOAD_POOL=${pool:-0} tools/mmsg_bench gpu 300 $extra \
          > $O/seam_${name}_$rep.json 2> $O/seam_${name}_$rep.err; rc=$?
      else
        timeout -k 10 120 tools/mmsg_bench cpu 300 > $O/seam_${name}_$rep.json 2> $O/seam_${name}_$rep.err; rc=$?
      fi
      echo "seam $name rep=$rep rc=$rc $(cat $O/seam_${name}_$rep.json) $(grep -o 'in_place=[0-9]* staged=[0-9]*' $O/seam_${name}_$rep.err)"
      ok_rc $rc || return $rc
    done
    for v in "rxplain:rx:" "rxdrop_staged:rx:gpu" "rxdrop_pool:rx:pool" "rxcpu:rxcpu:"; do
      IFS=: read name mode how <<< "$v"
      if [ -n "$how" ]; then
        local poolenv=TCPCSUM_PRELOAD_POOL=0
        [ "$how" = pool ] && poolenv=TCPCSUM_PRELOAD_POOL=mmsg_bench
        timeout -k 10 120 env LD_PRELOAD=$PRE TCPCSUM_PRELOAD_ANY_SOCKET=1 TCPCSUM_PRELOAD_TX=off \
          TCPCSUM_PRELOAD_RX=drop TCPCSUM_PRELOAD_STATS=1 $poolenv \
          tools/mmsg_bench $mode 300 > $O/seam_${name}_$rep.json 2> $O/seam_${name}_$rep.err; rc=$?
      else
        timeout -k 10 120 tools/mmsg_bench $mode 300 > $O/seam_${name}_$rep.json 2> $O/seam_${name}_$rep.err; rc=$?
      fi
      echo "seam $name rep=$rep rc=$rc $(cat $O/seam_${name}_$rep.json) $(grep -o 'in_place=[0-9]* staged=[0-9]*' $O/seam_${name}_$rep.err)"
      ok_rc $rc || return $rc
    done
  done
}

# wire FILL / VERIFY: the in-tree library against the round-3 and round-4 builds
# (tools/ab_build.sh), interleaved in one process, byte-identity checked
wire_ab() {
  WIRE_AB_ONLY=${WIRE_AB_ONLY:-1Mx1500_slots1536,1Mx1500_packed,128Kx9000_slots9216} WIRE_AB_ROUNDS=${1:-5} \
    timeout -k 10 400 python3 -u tools/wire_lib_ab.py tcp_amd/ab/libtcpcsum_wire_r3.so tcp_amd/ab/libtcpcsum_wire_r4.so \
    > $O/wire_ab.jsonl 2> $O/wire_ab.err; rc=$?
  cat $O/wire_ab.jsonl; return $rc
}

# the default bench line (driver form), plus $@ extra bench.py flags
bench() {
  timeout -k 10 900 python3 -u bench.py "$@" > $O/bench.json 2> $O/bench.err; rc=$?
  tail -c 600 $O/bench.err; python3 - << 'PY'
import json
d = json.load(open("gpurun_out/r5/bench.json"))
print("value", d["value"], "frac", d["roofline"]["frac"], "probe", d.get("stream_probe"))
oc = d.get("other_configs", {})
for k, v in oc.items():
    if k == "wire_1500":
        print(k, {m: v[m].get("kernel_avg_ms", v[m].get("avg_ms")) for m in ("fill", "verify", "copy_probe", "read_probe")},
              "fill/verify", v["fill_over_verify"], "fill/copy_probe", v["fill_over_copy_probe"], "check", v["check"])
    else:
        print(k, v["kernel_avg_ms"], v["roofline_frac"], v.get("stream_probe"), v.get("multi_batch", {}).get("roofline_frac"))
for m, v in (d.get("host_path") or {}).items():
    print("host", m, v["GiB/s"], v.get("raw_pinned_h2d_GiB/s"), v["cpu_core_s_per_step_rank0"], v["cgroup_throttled_ms_per_rank"],
          v["copy_threads_per_rank"], v["digest_check"])
print("cpu", d.get("cpu_baseline", {}).get("value"), "digest", d["digest_check"])
PY
  return $rc
}

# write-back probe shapes beside the wire FILL / VERIFY (tools/probe_rw_sweep.py)
probe_rw() {
  timeout -k 10 300 python3 -u tools/probe_rw_sweep.py > $O/probe_rw.jsonl 2> $O/probe_rw.err; rc=$?
  cat $O/probe_rw.jsonl; return $rc
}

# bench.py at N ranks on this one GPU (TCPCSUM_BENCH_SHARE_DEVICE=1): the launcher, barriers,
# every rank's shard digest, per-rank throttling and copy-thread budget — not the scaling
shared() {
  local n=${1:-8}
  TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 900 python3 -u bench.py --gpus $n --steps ${2:-20} --warmup 3 \
    > $O/bench_n${n}_shared.json 2> $O/bench_n${n}_shared.err; rc=$?
  tail -c 400 $O/bench_n${n}_shared.err; python3 - $n << 'PY'
import json, sys
d = json.load(open(f"gpurun_out/r5/bench_n{sys.argv[1]}_shared.json"))
print("n", d["n_gpus"], "value", d["value"], "digest", d["digest_check"])
for m, v in (d.get("host_path") or {}).items():
    print("host", m, v["GiB/s"], v["per_rank_GiB/s"], "throttled", v["cgroup_throttled_ms_per_rank"],
          "threads", v["copy_threads_per_rank"], "lws", v["local_world_size"], "digest", v["digest_check"])
PY
  return $rc
}

# 1M x 64-B batches: launch shapes of the uniform kernel beside the probe (tools/sweep.py)
sweep64() {
  timeout -k 10 600 python3 -u tools/sweep.py --config 64 --rounds 3 --steps 100 --probe \
    --blocks 512,1024,2048,4096,8192,16384,0 --unrolls 1,2,4,8 --shapes=-1,0,1,10,11 \
    > $O/sweep64.jsonl 2> $O/sweep64.err; rc=$?
  python3 -c "
import json
rows = [json.loads(l) for l in open('$O/sweep64.jsonl')]
for r in sorted((r for r in rows if 'med_ms' in r), key=lambda r: r['med_ms'])[:8]: print(r)
print([r for r in rows if 'probe_med_ms' in r or (r.get('shape') == -1 and r.get('max_blocks') == 0 and r.get('unroll') == 1)])
"; return $rc
}

# in-place host FILL of one releaseSend batch: store shape x kernel shape (tools/host_fill_ab.py)
host_fill() {
  timeout -k 10 300 python3 -u tools/host_fill_ab.py > $O/host_fill.jsonl 2> $O/host_fill.err; rc=$?
  cat $O/host_fill.jsonl; return $rc
}

# A/B of the in-tree library against tcp_amd/ab/$1/libtcpcsum.so on the seam (pool, staged) and
# the in-place host FILL, interleaved $2 times (the old library through LD_LIBRARY_PATH /
# TCPCSUM_LIB: mmsg_bench and the preload find libtcpcsum.so by RUNPATH, which it precedes)
lib_ab() {
  local old=$PWD/tcp_amd/ab/$1 reps=${2:-3}
  for rep in $(seq 1 $reps); do
    for which in new old; do
      local lp="" tl=""
      [ $which = old ] && lp=$old && tl=$old/libtcpcsum.so
      for v in pool staged; do
        local pool=0; [ $v = pool ] && pool=mmsg_bench
        timeout -k 10 120 env LD_LIBRARY_PATH=$lp LD_PRELOAD=$PRE TCPCSUM_PRELOAD_ANY_SOCKET=1 \
          TCPCSUM_PRELOAD_TX=fill TCPCSUM_PRELOAD_STATS=1 TCPCSUM_PRELOAD_POOL=$pool tools/mmsg_bench gpu 300 \
          > $O/libab_${which}_${v}_$rep.json 2> $O/libab_${which}_${v}_$rep.err || return $?
        echo "$which $v rep=$rep $(python3 -c "import json; d=json.load(open('$O/libab_${which}_${v}_$rep.json')); print(d['median_us'], d['min_us'], d['cpu_us_median'], d['checks_match_cpu'])") $(grep -o 'in_place=[0-9]*' $O/libab_${which}_${v}_$rep.err)"
      done
      env ${tl:+TCPCSUM_LIB=$tl} ROUNDS=2 timeout -k 10 200 python3 -u tools/host_fill_ab.py > $O/libab_${which}_hostfill_$rep.jsonl 2>> $O/libab.err || return $?
      echo "$which hostfill rep=$rep $(head -2 $O/libab_${which}_hostfill_$rep.jsonl | tr '\n' ' ')"
    done
  done
}

# the round's one rehearsal: every GPU test, smoke(), the default bench line, a rocprofv3
# kernel trace of the bench, and PMC passes (FETCH_SIZE of the headline; WRITE_SIZE and
# FETCH_SIZE of the wire FILL / VERIFY / write-back probe), each pass its own run
final() {
  export TMPDIR=/tmp
  tests || return $?
  cp $O/gputest.txt $O/gputest_final.txt
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; return 1; }
  tail -3 $O/smoke.txt
  bench || return $?
  cp $O/bench.json $O/bench_final.json
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python3 bench.py --no-host-path --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/rocprof.err || return $?
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_h -o fetch -- \
    python3 bench.py --steps 50 --no-other-configs --no-host-path --no-cpu-baseline > $O/pmc_h.json 2> $O/pmc_h.err || return $?
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o write -- \
    python3 tools/wire_fill_pmc.py > $O/pmc_w.txt 2> $O/pmc_w.err || return $?
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o fetch -- \
    python3 tools/wire_fill_pmc.py > $O/pmc_f.txt 2> $O/pmc_f.err || return $?
  find $O/prof $O/pmc_h $O/pmc_w $O/pmc_f -name "*.csv" | head -20
  # last: round 4's exit-time SIGSEGV record (gpurun_out/r4_hostprof.err) — the same command again
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/hostprof -o h -- \
    python3 bench.py --host-path-only --host-steps 5 > $O/hostprof.json 2> $O/hostprof.err
  echo "hostprof rc=$?"
}

# round 4's exit-time SIGSEGV under rocprofv3 --memory-copy-trace, with the process's address map
# saved at exit (tools/maps_at_exit.py) so the faulting frames can be resolved to libraries
hostprof_maps() {
  export TMPDIR=/tmp MAPS_OUT=$O/maps_at_exit.txt
  timeout -k 10 300 rocprofv3 ${@:---kernel-trace --memory-copy-trace} --output-format csv -d $O/hostprof2 -o h -- \
    python3 tools/maps_at_exit.py bench.py --host-path-only --host-steps 5 > $O/hostprof2.json 2> $O/hostprof2.err
  local rc=$?
  cp /proc/self/maps $O/maps_shell.txt 2>/dev/null
  echo "hostprof rc=$rc"; tail -20 $O/hostprof2.err
}

"$@"
