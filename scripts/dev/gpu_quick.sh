#!/bin/bash
# Quick GPU check of a change: selected kernel tests, the model parity tests, one bench line.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
K="${K:-a3_bwd or conv_bwd}"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "$K" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
if [ "${PARITY:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
  tail -2 gpurun_out/t2.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b1.log 2>&1 || { tail -20 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log | cut -c1-220
