#!/bin/bash
# Round 4: class-row to_out forward on 2-column workgroups -- parity / interface
# tests, then kernel traces against ab/ (the previous commit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 700 $T tests/test_parity_gpu.py tests/test_interface.py \
  > gpurun_out/r04ee_t.log 2>&1 || { tail -40 gpurun_out/r04ee_t.log; exit 1; }
tail -1 gpurun_out/r04ee_t.log
AB_PAIRS=3 bash scripts/dev/ab_prof.sh || exit 1
python3 scripts/dev/trace_diff.py "gpurun_out/prof_A*" "gpurun_out/prof_B*" > gpurun_out/r04ee_diff.txt 2>&1
head -12 gpurun_out/r04ee_diff.txt; grep -i "cls_out_fwd\|total" gpurun_out/r04ee_diff.txt
