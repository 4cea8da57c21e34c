#!/bin/bash
# round 6, first session: the changed GPU tests, the driver's bench command next to a 200-step run,
# then the RCCL teardown diagnostic (old order last: it may abort the process)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06a
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_ddp_gpu.py tests/test_bench_gpu.py tests/test_parity_gpu.py -k "ddp or two_rank or rccl or bench or bf16_mode_close or fused_backward" \
  > "$OUT/tests.txt" 2>&1
rc=$?; tail -3 "$OUT/tests.txt"
[ $rc -eq 0 ] || { echo "tests rc=$rc: stopping"; exit $rc; }
echo "== bench 20 $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench20.log" 2>&1
rc=$?; tail -1 "$OUT/bench20.log" | cut -c1-300
[ $rc -eq 0 ] || exit $rc
echo "== bench 200 $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/bench200.log" 2>&1
rc=$?; tail -1 "$OUT/bench200.log" | cut -c1-300
[ $rc -eq 0 ] || exit $rc
echo "== bench 20 again $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-hbm-probe > "$OUT/bench20b.log" 2>&1
rc=$?; tail -1 "$OUT/bench20b.log" | cut -c1-300
[ $rc -eq 0 ] || exit $rc
echo "== rccl teardown close $(date +%T)"
timeout -k 10 200 python -u scripts/dev/rccl_teardown.py close > "$OUT/rccl_close.txt" 2>&1
rc=$?; tail -2 "$OUT/rccl_close.txt"
[ $rc -eq 0 ] || exit $rc
echo "== rccl teardown old $(date +%T)"
NCCL_DEBUG=WARN timeout -k 10 200 python -u scripts/dev/rccl_teardown.py old > "$OUT/rccl_old.txt" 2>&1
rc=$?; tail -4 "$OUT/rccl_old.txt"; echo "old rc=$rc"
exit 0
