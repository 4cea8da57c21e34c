#!/bin/bash
# HBM traffic of the bench's probed kernel from rocprofv3 PMC counters: one pass per
# counter (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), kernel-trace only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_$C -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc_$C.log 2>&1 || exit $?
done
python3 scripts/traffic_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE ${KERNELS:-a1_fwd_kernel}
