#!/bin/bash
# Round 4: optimizer with per-workgroup step counters (no tick launch) + assemble_q_slab unroll:
# the optimizer / interface / sibling / bench-step tests, then a bench line and kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_interface.py tests/test_siblings_gpu.py tests/test_bench_gpu.py tests/test_kernels_gpu.py -k "radam or optim or bench or assemble or sibling or task" \
  > gpurun_out/r04g_t.log 2>&1 || { tail -30 gpurun_out/r04g_t.log; exit 1; }
tail -2 gpurun_out/r04g_t.log
PARITY=0 K=assemble PROF=1 bash scripts/gpu_quick2.sh
