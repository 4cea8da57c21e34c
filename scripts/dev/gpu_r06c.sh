set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-hbm-probe > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-hbm-probe > $OUT/prof_bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/prof_bench.log; exit $rc; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python scripts/dev/trace_gaps.py "$f" --top 60 > $OUT/gaps.txt 2>&1; head -50 $OUT/gaps.txt
