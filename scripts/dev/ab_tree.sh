#!/bin/bash
# A/B of the working tree against a git revision on ONE box.
#   bash scripts/dev/ab_tree.sh prepare [REV]   (here: exports REV (default HEAD) to ab/ and builds its library)
#   bash scripts/dev/ab_tree.sh run             (on the box: alternates bench.py of the tree (A) and of ab/ (B))
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
if [ "${1:-}" = "prepare" ]; then
  rm -rf ab && mkdir ab && git archive "${2:-HEAD}" | tar -x -C ab && make -C ab/transmil_deepgraft_amd/csrc -j8 > /dev/null && rm -rf ab/tests ab/profiles ab/transmil_deepgraft_amd/csrc/build
  exit $?
fi
for i in $(seq ${AB_PAIRS:-3}); do
  for tag in A B; do
    dir=.; [ $tag = B ] && dir=ab
    (cd $dir && timeout -k 10 300 python bench.py --steps ${AB_STEPS:-300} --warmup 10 --no-cpu-baseline --no-hbm-probe ${BENCH_ARGS:-} 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'])") || exit 1
  done
done
