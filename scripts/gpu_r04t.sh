#!/bin/bash
# Round 4: kernel traces of the C5 train-BN and eval steps (MIOpen find on), after the BN fixes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in train eval; do
  timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/c5$mode -o run --output-format csv -- \
    python3 scripts/bench_c5.py --encoder-mode $mode --steps 2 --warmup 1 > gpurun_out/r04t_$mode.log 2>&1 || { tail -20 gpurun_out/r04t_$mode.log; exit 1; }
  tail -1 gpurun_out/r04t_$mode.log | cut -c1-200
done
