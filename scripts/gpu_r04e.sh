#!/bin/bash
# Round 4: fused train-mode BN encoder at growing bag sizes (stop at the first failure), then the
# C5 bench in both modes + eval kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoder.py -x -v --timeout 300 --timeout-method thread -m gpu -k "conv1x1 or bn_train or train_mode" \
  > gpurun_out/r04e_enc.log 2>&1 || { tail -40 gpurun_out/r04e_enc.log; exit 1; }
tail -1 gpurun_out/r04e_enc.log
for n in 1024 4096; do
  timeout -k 10 300 python scripts/bench_c5.py --n $n --steps 2 --warmup 1 --encoder-mode train \
    > gpurun_out/c5_r04e_train_$n.log 2>&1 || { tail -30 gpurun_out/c5_r04e_train_$n.log; exit 1; }
  tail -1 gpurun_out/c5_r04e_train_$n.log | cut -c1-300
done
TAG=r04e bash scripts/gpu_c5.sh
