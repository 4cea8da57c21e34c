#!/bin/bash
# One measurement session on the GPU box: the default bench line, a kernel trace + stats of a
# short bench, and the PMC passes (each step under its own time limit; the first failure ends it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python3 scripts/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv 16 40 > gpurun_out/${TAG}_kernel_summary.txt
python3 scripts/chain_summary.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_pinv_chain.json
head -12 gpurun_out/${TAG}_kernel_summary.txt; cat gpurun_out/${TAG}_pinv_chain.json
if [ "${PMC:-1}" = "1" ]; then
  PMC_OUT=gpurun_out/${TAG}_pmc PASSES="${PASSES:-sq tcc fetch write}" bash scripts/gpu_pmc_bench.sh || exit $?
  python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc --top 14 > gpurun_out/${TAG}_pmc.json
fi
echo measure done
