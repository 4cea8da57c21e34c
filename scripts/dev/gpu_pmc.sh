#!/bin/bash
# rocprofv3 PMC counters (kernel trace only, no other tracing) for one microbench case.
#   CASE="gemm qkv (NT" COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY ..." bash scripts/dev/gpu_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
timeout -k 10 600 rocprofv3 --kernel-trace --pmc ${COUNTERS} -d "$OUT" -o run --output-format csv -- \
  python3 scripts/microbench.py --only "${CASE}" --reps ${REPS:-5} > gpurun_out/pmc_bench.log 2>&1
rc=$?
echo "rocprof pmc rc=$rc"; tail -3 gpurun_out/pmc_bench.log
exit $rc
