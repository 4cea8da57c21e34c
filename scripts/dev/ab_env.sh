#!/bin/bash
# A/B of two environments on ONE box with the same tree: bench.py alternated, A = $AB_ENV_A, B = $AB_ENV_B
# (e.g. AB_ENV_A="" AB_ENV_B="TM_GEMM_QKV_BIG=0")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for i in $(seq ${AB_PAIRS:-4}); do
  for tag in A B; do
    envs=${AB_ENV_A:-}; [ $tag = B ] && envs=${AB_ENV_B:-}
    env $envs timeout -k 10 300 python bench.py --steps ${AB_STEPS:-300} --warmup 10 --no-cpu-baseline --no-hbm-probe 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'])" || exit 1
  done
done
