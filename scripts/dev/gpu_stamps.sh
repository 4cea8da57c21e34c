#!/bin/bash
# Diagnostic build stamp runs (libtransmil_hip_diag.so): per-phase s_memtime of the A3 forward and
# backward at the bench shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/dev/a3_fwd_stamps.py > gpurun_out/st_a3f.log 2>&1 || { tail -20 gpurun_out/st_a3f.log; exit 1; }
cat gpurun_out/st_a3f.log
A3_STAMPS=30 timeout -k 10 120 python scripts/dev/a3_bwd_stamps.py > gpurun_out/st_a3b30.log 2>&1 || { tail -20 gpurun_out/st_a3b30.log; exit 1; }
cat gpurun_out/st_a3b30.log
A3_STAMPS=31 timeout -k 10 120 python scripts/dev/a3_bwd_stamps.py > gpurun_out/st_a3b31.log 2>&1 || { tail -20 gpurun_out/st_a3b31.log; exit 1; }
cat gpurun_out/st_a3b31.log
