#!/bin/bash
# One GPU session of named stages (STAGES="tests bench prof c5drift c5 pmc"), each under its own
# time limit; the first failing stage ends the script (no retries).  Outputs under gpurun_out/$TAG/.
#   tests    pytest -m gpu (TESTS= to select)                 -> gpu_tests.txt
#   smoke    __graft_entry__.smoke()                            -> smoke.txt
#   bench    bench.py (BENCH_ARGS=, default: no CPU baseline)  -> bench.log
#   prof     rocprofv3 --kernel-trace --stats of the bench      -> prof/
#   c5drift  scripts/dev/c5_drift.py under a kernel trace       -> c5_drift.json, c5drift_prof/
#   c5       scripts/bench_c5.py (C5_ARGS=)                      -> c5.log
#   pmc      PMC passes over the bench (scripts/gpu_pmc_bench.sh) -> pmc/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {   # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stopping"; exit $rc; fi
}
for S in ${STAGES:-tests bench}; do
  case $S in
    tests)
      run tests 900 bash -c "python -u -m pytest ${TESTS:-tests} -v -m gpu -p no:cacheprovider --timeout 150 \
        --timeout-method thread > $OUT/gpu_tests.txt 2>&1"
      tail -2 "$OUT/gpu_tests.txt" ;;
    smoke)
      run smoke 300 bash -c "python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > $OUT/smoke.txt 2>&1"
      tail -1 "$OUT/smoke.txt" ;;
    bench)
      run bench 600 bash -c "python -u bench.py ${BENCH_ARGS:---no-cpu-baseline --no-cpu-as-written} > $OUT/bench.log 2>&1"
      tail -1 "$OUT/bench.log" | cut -c1-300 ;;
    prof)
      run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-cpu-as-written --steps ${PROF_STEPS:-200} > "$OUT/prof_bench.log" 2>&1
      tail -1 "$OUT/prof_bench.log" | cut -c1-200 ;;
    c5drift)
      run c5drift 600 rocprofv3 --kernel-trace --stats -d "$OUT/c5drift_prof" -o run --output-format csv -- \
        python3 scripts/dev/c5_drift.py > "$OUT/c5_drift.json" 2> "$OUT/c5_drift.log"
      tail -3 "$OUT/c5_drift.log" ;;
    c5)
      run c5 900 bash -c "python -u scripts/bench_c5.py ${C5_ARGS:-} > $OUT/c5.log 2>&1"
      tail -2 "$OUT/c5.log" | cut -c1-400 ;;
    pmc)
      run pmc 900 env PMC_OUT="$OUT/pmc" PASSES="${PASSES:-sq tcc fetch write}" bash scripts/gpu_pmc_bench.sh
      ;;
    *) echo "unknown stage $S"; exit 2 ;;
  esac
done
echo "session done"
