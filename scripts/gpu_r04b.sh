#!/bin/bash
# Round-4 GPU pass 2: the C5 test, the rest of the suite, the bench, then C5 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_encoder.py tests/test_interface.py tests/test_ddp_gpu.py > gpurun_out/r04b_new.log 2>&1
rc=$?; tail -25 gpurun_out/r04b_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $T tests --deselect tests/test_encoder.py::test_c5_full_bag_4096_tiles > gpurun_out/r04b_all.log 2>&1
rc=$?; tail -5 gpurun_out/r04b_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r04b_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r04b_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
PROF=0 bash scripts/gpu_c5.sh
