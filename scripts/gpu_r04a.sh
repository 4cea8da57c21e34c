#!/bin/bash
# Round-4 first GPU pass: the new / changed tests, then the full GPU suite, then the bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_reentrant_gpu.py tests/test_encoder.py tests/test_interface.py tests/test_ddp_gpu.py > gpurun_out/r04a_new.log 2>&1
rc=$?; tail -25 gpurun_out/r04a_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $T tests > gpurun_out/r04a_all.log 2>&1
rc=$?; tail -5 gpurun_out/r04a_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r04a_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r04a_bench.log | cut -c1-300; exit $rc
