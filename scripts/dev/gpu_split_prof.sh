#!/bin/bash
# split pinv: tests, ablation microbench, and a kernel trace of the split forward / backward
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pinv_split_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_split.log 2>&1
rc=$?; tail -3 gpurun_out/t_split.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python scripts/microbench.py --only "pinv" --reps 10 > gpurun_out/mb_pinv3.log 2>&1 || exit $?
cat gpurun_out/mb_pinv3.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split -o run --output-format csv -- python3 scripts/microbench.py --only "pinv_fwd split [full]" --reps 10 > gpurun_out/prof_split.log 2>&1 || exit $?
python3 scripts/prof_summary.py $(ls gpurun_out/prof_split/*/run_kernel_stats.csv gpurun_out/prof_split/run_kernel_stats.csv 2>/dev/null | head -1) 1 12
