#!/bin/bash
# Full GPU suite, smoke, bench (with CPU baseline), then the C5 bench lines + the bench rocprof.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 1000 $T tests > gpurun_out/r04c_all.log 2>&1
rc=$?; tail -4 gpurun_out/r04c_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04c_smoke.log 2>&1 || { tail -5 gpurun_out/r04c_smoke.log; exit 1; }
tail -1 gpurun_out/r04c_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r04c_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r04c_bench.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
PROF=1 TAG=r04c bash scripts/gpu_c5.sh
