#!/bin/bash
# rocprofv3 PMC passes over a short bench run: one pass per counter group (kernel trace only,
# no other tracing), each under its own SIGKILL time limit; the first failing pass ends the script.
#   PASSES="sq tcc fetch write" BENCH_ARGS="--n 8192" bash scripts/gpu_pmc_bench.sh
# then: python3 scripts/pmc_summary.py gpurun_out/pmc > profiles/<name>.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
declare -A GROUP
GROUP[sq]="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
GROUP[tcc]="TCC_HIT_sum TCC_MISS_sum"
GROUP[fetch]="FETCH_SIZE"
GROUP[write]="WRITE_SIZE"
GROUP[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for P in ${PASSES:-sq tcc fetch write}; do
  echo "pass $P: ${GROUP[$P]}"
  timeout -s KILL ${PASS_TIMEOUT:-150} rocprofv3 --kernel-trace --pmc ${GROUP[$P]} -d "$OUT/$P" -o run --output-format csv -- \
    python3 bench.py --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "gpurun_out/pmc_$P.log" 2>&1
  rc=$?
  tail -2 "gpurun_out/pmc_$P.log"
  if [ $rc -ne 0 ]; then echo "pass $P rc=$rc: stopping"; exit $rc; fi
done
echo "pmc passes done"
