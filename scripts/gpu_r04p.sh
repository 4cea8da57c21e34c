#!/bin/bash
# Round 4: C5 with MIOpen find (torch.backends.cudnn.benchmark) against the default immediate mode,
# eval-BN and train-BN encoder, 4096 tiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in eval train; do
  for b in "" "--benchmark"; do
    timeout -k 10 400 python -u scripts/bench_c5.py --encoder-mode $mode --steps 4 --warmup 2 $b \
      > gpurun_out/r04p_${mode}${b}.log 2>&1 || { tail -20 gpurun_out/r04p_${mode}${b}.log; exit 1; }
    tail -1 gpurun_out/r04p_${mode}${b}.log | cut -c1-420
  done
done
