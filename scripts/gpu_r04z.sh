#!/bin/bash
# Round 4: eager host-path A/B (working tree A vs ab/ = previous commit B) on one box, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for tag in A B; do
    dir=.; [ $tag = B ] && dir=ab
    (cd $dir && timeout -k 10 300 python -u $OLDPWD/scripts/dev/graphed_step_rate.py 2>/dev/null | tail -1 | sed "s/^/$tag /") || exit 1
  done
done
