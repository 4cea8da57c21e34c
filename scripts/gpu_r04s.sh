#!/bin/bash
# Round 4: the BatchNorm statistics partial pass as one launch over all pieces -- encoder tests,
# then the C5 train-BN and eval steps (MIOpen find on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 700 $T tests/test_encoder.py > gpurun_out/r04s_t.log 2>&1 || { tail -40 gpurun_out/r04s_t.log; exit 1; }
tail -1 gpurun_out/r04s_t.log
for mode in train eval; do
  timeout -k 10 400 python -u scripts/bench_c5.py --encoder-mode $mode --steps 4 --warmup 2 \
    > gpurun_out/r04s_$mode.log 2>&1 || { tail -20 gpurun_out/r04s_$mode.log; exit 1; }
  tail -1 gpurun_out/r04s_$mode.log | cut -c1-200
done
