#!/bin/bash
# Round 4: bench with K = 10 gradient accumulation (C4's all-reduce-every-10-steps row, one GPU) and
# the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 40 --warmup 3 --accumulate 10 --no-cpu-baseline --no-hbm-probe \
  > gpurun_out/r04f_acc10.log 2>&1 || { tail -30 gpurun_out/r04f_acc10.log; exit 1; }
tail -1 gpurun_out/r04f_acc10.log | cut -c1-700
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-hbm-probe > gpurun_out/r04f_acc1.log 2>&1 || { tail -30 gpurun_out/r04f_acc1.log; exit 1; }
tail -1 gpurun_out/r04f_acc1.log | cut -c1-400
