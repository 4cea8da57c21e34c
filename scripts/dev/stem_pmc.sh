#!/bin/bash
# PMC passes (HBM bytes, MFMA activity) of the C5 stem kernel under scripts/dev/stem_time.py, then a 1000-step bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05stem
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/r05stem/$tag -o run --output-format csv -- python3 scripts/dev/stem_time.py 1024 > gpurun_out/r05stem/$tag.log 2>&1 || exit $?
done
timeout -k 10 400 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-cpu-as-written > gpurun_out/r05stem/bench1000.log 2>&1
