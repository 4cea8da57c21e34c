#!/bin/bash
# rocprofv3 kernel traces of the working tree (A) and ab/ (B) on ONE box, alternated A B A B
# (bench, 40 steps each); compare with scripts/dev/trace_diff.py (per-kernel min over the runs).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq ${AB_PAIRS:-2}); do
  for tag in A B; do
    dir=.; [ $tag = B ] && dir=ab
    (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_$tag$i" -o run --output-format csv -- \
       python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-hbm-probe > "$ROOT/gpurun_out/prof_$tag$i.log" 2>&1) || exit 1
    tail -1 "gpurun_out/prof_$tag$i.log" | cut -c1-100
  done
done
