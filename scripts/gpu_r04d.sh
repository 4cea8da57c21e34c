#!/bin/bash
# Round 4: encoder tests (fused 1x1 epilogue, bias+ReLU pass, train-mode whole-bag BN), then the C5
# bench in both encoder modes + a kernel trace of the eval run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoder.py -x -v --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/r04d_enc.log 2>&1 || { tail -40 gpurun_out/r04d_enc.log; exit 1; }
tail -3 gpurun_out/r04d_enc.log
TAG=r04d bash scripts/gpu_c5.sh
