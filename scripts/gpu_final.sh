#!/bin/bash
# Round-end evidence in ONE GPU session, every step under its own time limit; the first failing
# step ends the script (no retries):
#   1. the GPU test suite            -> gpurun_out/final/gpu_tests.txt
#   2. __graft_entry__.smoke()       -> gpurun_out/final/smoke.txt
#   3. bench.py as the driver runs it (default flags: CPU baselines + hbm_roofline probe)
#                                    -> gpurun_out/final/bench.log
#   3b. bench.py --gpus 1 --steps 20 --warmup 5 (the driver's exact command)
#                                    -> gpurun_out/final/bench_driver_cmd.log
#   4. rocprofv3 --kernel-trace --stats of the same bench command (no PMC here)
#                                    -> gpurun_out/final/prof/
#   5. PMC passes (SQ, TCC, FETCH_SIZE, WRITE_SIZE), one counter group per run
#                                    -> gpurun_out/pmc/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step tests
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"
[ $rc -eq 0 ] || { echo "tests rc=$rc: stopping"; exit $rc; }
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
rc=$?; tail -2 "$OUT/smoke.txt"
[ $rc -eq 0 ] || { echo "smoke rc=$rc: stopping"; exit $rc; }
step bench
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log" | cut -c1-200
[ $rc -eq 0 ] || { echo "bench rc=$rc: stopping"; exit $rc; }
step bench-driver-command
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_cmd.log" 2>&1
rc=$?; tail -1 "$OUT/bench_driver_cmd.log" | cut -c1-200
[ $rc -eq 0 ] || { echo "bench (driver command) rc=$rc: stopping"; exit $rc; }
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-cpu-as-written > "$OUT/prof_bench.log" 2>&1
rc=$?; tail -1 "$OUT/prof_bench.log" | cut -c1-200
[ $rc -eq 0 ] || { echo "rocprof rc=$rc: stopping"; exit $rc; }
step pmc
PASSES="sq tcc fetch write" bash scripts/gpu_pmc_bench.sh > "$OUT/pmc.log" 2>&1
rc=$?; tail -1 "$OUT/pmc.log"
exit $rc
