#!/bin/bash
# rocprofv3 kernel traces of the working tree (A) and ab/ (B) on ONE box (bench, 40 steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in A B; do
  dir=.; [ $tag = B ] && dir=ab
  (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$tag" -o run --output-format csv -- \
     python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-hbm-probe > "$GRAFT_REPO_ROOT/gpurun_out/prof_$tag.log" 2>&1) || exit 1
  tail -1 "gpurun_out/prof_$tag.log" | cut -c1-120
done
