#!/usr/bin/env bash
# Round-6 GPU runs, one function per experiment; outputs under gpurun_out/r6/:
#   bash tools/r6_runs.sh <function> [args] [-- <function> [args] ...]
# Several functions may be chained with "--"; the first failure ends the call.
# Every GPU step runs under its own timeout.
set -o pipefail
O=gpurun_out/r6
mkdir -p $O
export TMPDIR=/tmp

# GPU tests of the files named (default: all), one pytest process
tests() {
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "${@:-tests}" \
    > $O/gputest.txt 2>&1; local rc=$?
  tail -5 $O/gputest.txt; return $rc
}

smoke() {
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; local rc=$?
  tail -3 $O/smoke.txt; return $rc
}

# bench.py exactly as the driver runs it (python3 bench.py --gpus 1 --steps 20 --warmup 5), or with
# the flags given; output $O/bench_<tag>.json, tag = $BTAG or "driver"
bench() {
  local tag=${BTAG:-driver}
  local args=("$@"); [ ${#args[@]} = 0 ] && args=(--gpus 1 --steps 20 --warmup 5)
  timeout -k 10 600 python3 -u bench.py "${args[@]}" > $O/bench_$tag.json 2> $O/bench_$tag.err; local rc=$?
  tail -c 400 $O/bench_$tag.err
  python3 tools/bench_summary.py $O/bench_$tag.json
  return $rc
}

# run length / first read / probe order on the 64-B and 1500-B configs (tools/runlen_ab.py)
runlen() {
  timeout -k 10 600 python3 -u tools/runlen_ab.py > $O/runlen.jsonl 2> $O/runlen.err; local rc=$?
  cat $O/runlen.jsonl; tail -5 $O/runlen.err; return $rc
}

# any python tool under tools/ with its args: output $O/<name>.jsonl
py() {
  local name=$(basename $1 .py)
  timeout -k 10 ${PYT:-600} python3 -u "$@" > $O/$name.jsonl 2> $O/$name.err; local rc=$?
  cat $O/$name.jsonl; tail -5 $O/$name.err; return $rc
}

# uniform kernel shapes -1 (the plan), 13 (split) and 14 (workgroup per segment) x unroll at
# each length given (default: the long-segment sizes), ~1.5 GB batches: $O/sweeplens.jsonl
sweeplens() {
  [ $# -gt 0 ] && LENS="$*"
  : > $O/sweeplens.jsonl
  for L in ${LENS:-8192 9000 12300 16384 20004 32768 65536 131072}; do
    timeout -k 10 300 python3 -u tools/sweep.py --len $L --shapes=-1,13,14 --blocks 0 --unrolls 1,2,4,8 \
      --rounds 3 --steps 20 >> $O/sweeplens.jsonl 2>> $O/sweeplens.err || return $?
  done
  python3 - << 'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6/sweeplens.jsonl") if l.strip()]
by = collections.defaultdict(list)
for r in rows: by[r["config"]].append(r)
for c, rs in by.items():
    rs.sort(key=lambda r: r["med_ms"])
    plan = [r for r in rs if r["shape"] == -1 and r["unroll"] == 1]
    print(c, "best", [(r["shape"], r["unroll"], r["med_ms"], r["same_results"]) for r in rs[:3]],
          "plan(u1)", [(r["med_ms"]) for r in plan], "all_same", all(r["same_results"] for r in rs))
PY
}

# rocprofv3 kernel trace + stats of the driver's bench command
prof() {
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-host-path --no-cpu-baseline --no-seam \
    > $O/bench_under_rocprof.json 2> $O/rocprof.err; local rc=$?
  tail -3 $O/rocprof.err; return $rc
}

# one PMC pass (counters $1) over the bench with flags $2...: $O/pmc_<tag>/
pmc() {
  local ctr=$1; shift
  local tag=${PTAG:-$ctr}
  timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$tag -o pmc -- python3 "$@" \
    > $O/pmc_$tag.out 2> $O/pmc_$tag.err; local rc=$?
  tail -2 $O/pmc_$tag.err; return $rc
}

# bench.py at N ranks on this one GPU (TCPCSUM_BENCH_SHARE_DEVICE=1): the launcher, barriers,
# every rank's shard digest, per-rank throttling and copy-thread budget — not the scaling
shared() {
  local n=${1:-8}
  TCPCSUM_BENCH_SHARE_DEVICE=1 timeout -k 10 900 python3 -u bench.py --gpus $n --steps ${2:-20} --warmup 3 \
    > $O/bench_n${n}_shared.json 2> $O/bench_n${n}_shared.err; local rc=$?
  tail -c 400 $O/bench_n${n}_shared.err
  python3 tools/bench_summary.py $O/bench_n${n}_shared.json
  return $rc
}

# the round's one closing rehearsal, the driver's own commands: every GPU test, smoke(), the
# bench as the driver runs it, then the same bench under rocprofv3 --kernel-trace --stats, and
# the PMC passes, each its own run: FETCH_SIZE of the headline, 64 KiB and 64-B configs (the
# probe in each pass calibrates it), FETCH_SIZE / WRITE_SIZE of the wire FILL / VERIFY on MTU
# packets and on the flush mix
final() {
  tests || return $?
  smoke || return $?
  bench || return $?
  prof || return $?
  python3 tools/trace_runs.py $O/prof/bench_kernel_trace.csv > $O/trace_runs.jsonl
  local common="--gpus 1 --warmup 5 --no-other-configs --no-host-path --no-cpu-baseline --no-seam"
  PTAG=fetch_1500 pmc FETCH_SIZE bench.py --steps 20 $common || return $?
  PTAG=fetch_64k pmc FETCH_SIZE bench.py --config 64k --steps 10 $common || return $?
  PTAG=fetch_64 pmc FETCH_SIZE bench.py --config 64 --steps 50 $common || return $?
  PTAG=write_wire pmc WRITE_SIZE tools/wire_fill_pmc.py || return $?
  PTAG=fetch_wire pmc FETCH_SIZE tools/wire_fill_pmc.py || return $?
  PTAG=fetch_mix pmc FETCH_SIZE tools/wire_mix_pmc.py || return $?
  PTAG=write_mix pmc WRITE_SIZE tools/wire_mix_pmc.py || return $?
  ls $O/pmc_*/
}

# run the chained functions: f1 args -- f2 args -- ...
cmd=()
for a in "$@"; do
  if [ "$a" = "--" ]; then
    "${cmd[@]}" || exit $?
    cmd=()
  else
    cmd+=("$a")
  fi
done
[ ${#cmd[@]} -gt 0 ] && { "${cmd[@]}" || exit $?; }
exit 0
