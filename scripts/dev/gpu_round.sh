#!/bin/bash
# One GPU session: tests, then (only if no crash) a short bench.  Every GPU step
# has its own time limit; a crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TESTS="${TESTS:-tests}"
timeout -k 10 900 python -u -m pytest $TESTS -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -5 gpurun_out/bench.log
  exit $brc
fi
exit $rc
