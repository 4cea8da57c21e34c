#!/bin/bash
# Round 4: kernel statistics of the C5 train-BN step (MIOpen find on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/c5train -o run --output-format csv -- \
  python3 scripts/bench_c5.py --encoder-mode train --steps 2 --warmup 1 > gpurun_out/r04q.log 2>&1 || { tail -20 gpurun_out/r04q.log; exit 1; }
tail -1 gpurun_out/r04q.log | cut -c1-300
f=$(ls gpurun_out/c5train/*kernel_stats.csv | head -1)
head -25 "$f" | cut -d, -f1-5
