#!/usr/bin/env bash
# Build the library as it was at a git revision, for same-process A/B runs against
# the in-tree build (tools/wire_lib_ab.py, tools/lb_ab.py ...):
#   bash tools/ab_build.sh <rev> <name> [extra compiler flags]  ->  tcp_amd/ab/libtcpcsum_<name>.so
# Extra flags set measurement knobs, e.g. -DTCPCSUM_MEASUREMENT_BUILD=1 -DTCPCSUM_LINE_CPOL=2.
# (CPU only: hipcc cross-compiles gfx950 here; the .so travels with the tree.)
set -euo pipefail
rev=$1; name=$2; shift 2
extra=("$@")
src=$(mktemp -d)
trap 'rm -rf "$src"' EXIT
git archive "$rev" tcp_amd/csrc include | tar -x -C "$src"
mkdir -p tcp_amd/ab
objs=()
for f in "$src"/tcp_amd/csrc/*.hip; do
  o="$src/$(basename "$f" .hip).o"
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-value -Wno-unused-result "${extra[@]}" -I"$src/include" -c "$f" -o "$o" &
  objs+=("$o")
done
for f in "$src"/tcp_amd/csrc/*.c; do
  case $(basename "$f") in preload_*) continue ;; esac
  o="$src/$(basename "$f" .c).o"
  gcc -O2 -fPIC -I"$src/include" -c "$f" -o "$o"
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "tcp_amd/ab/libtcpcsum_$name.so" "${objs[@]}" -lpthread
echo "tcp_amd/ab/libtcpcsum_$name.so from $(git rev-parse --short "$rev")"
