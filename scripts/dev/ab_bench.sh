#!/bin/bash
# A/B of two builds on ONE box: bench.py with the in-tree library and with $AB_LIB, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for i in 1 2; do
  for lib in "" "$AB_LIB"; do
    if [ -n "$lib" ]; then export TRANSMIL_HIP_LIB=$lib; tag=B; else unset TRANSMIL_HIP_LIB; tag=A; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'])" || exit 1
  done
done
