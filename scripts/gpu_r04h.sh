#!/bin/bash
# Round 4 A/B: working tree (radam 4 pieces per thread, A3 backward dQ roles off SIMD 0) vs ab/ (HEAD)
# kernel traces, after the assemble_q_slab / optimizer / parity tests on the working tree; then C1 / C3 / 2048.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_interface.py tests/test_siblings_gpu.py tests/test_parity_gpu.py \
  > gpurun_out/r04h_t.log 2>&1 || { tail -30 gpurun_out/r04h_t.log; exit 1; }
tail -1 gpurun_out/r04h_t.log
AB_PAIRS=2 bash scripts/dev/ab_prof.sh || exit 1
python3 scripts/dev/trace_diff.py "gpurun_out/prof_A*" "gpurun_out/prof_B*" > gpurun_out/r04h_diff.txt 2>&1
head -40 gpurun_out/r04h_diff.txt
bash scripts/dev/bench_configs.sh
