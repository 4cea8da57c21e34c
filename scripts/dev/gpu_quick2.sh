#!/bin/bash
# Quick GPU check: selected kernel tests (K), the whole-model parity tests, one bench line (+ rocprof
# kernel stats when PROF=1).  Every GPU step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py -k "${K:-ppeg}" > gpurun_out/q_k.log 2>&1 || { tail -30 gpurun_out/q_k.log; exit 1; }
tail -2 gpurun_out/q_k.log
if [ "${PARITY:-1}" = "1" ]; then
  timeout -k 10 500 $T tests/test_parity_gpu.py > gpurun_out/q_p.log 2>&1 || { tail -30 gpurun_out/q_p.log; exit 1; }
  tail -2 gpurun_out/q_p.log
fi
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q_b.log 2>&1 || { tail -20 gpurun_out/q_b.log; exit 1; }
tail -1 gpurun_out/q_b.log | cut -c1-200
python - <<'PY'
import json
d = json.loads(open("gpurun_out/q_b.log").read().strip().splitlines()[-1])
for h in d.get("hbm_roofline") or []:
    print(f"  {h['site']}:{h['layer']} {h['us']} us frac {h['frac']}")
for k in ("roofline", "roofline_pinv_bwd"):
    r = d.get(k)
    if r: print(f"  {k}: {r['kernel_ms']} ms frac {r['frac']}")
PY
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hbm-probe > gpurun_out/qprof.log 2>&1 || { tail -5 gpurun_out/qprof.log; exit 1; }
  python3 scripts/prof_summary.py $(find gpurun_out/qprof -name "*kernel_stats.csv" | head -1) 27 30 > gpurun_out/qprof_summary.txt
  head -32 gpurun_out/qprof_summary.txt
fi
