#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench.log
find "$OUT" -name "*stats*" | head
exit $rc
