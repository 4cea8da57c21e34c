#!/bin/bash
# Round 4: C5 piece size 1024 (the size a whole 1024-tile bag ran at before) (tiles per encoder piece), eval and train BN, MIOpen find on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "eval 1024" "train 1024"; do
  set -- $cfg
  timeout -k 10 400 python -u scripts/bench_c5.py --encoder-mode $1 --chunk $2 --steps 3 --warmup 2 \
    > gpurun_out/r04v_$1_$2.log 2>&1 || { tail -20 gpurun_out/r04v_$1_$2.log; exit 1; }
  echo "$1 $2 $(tail -1 gpurun_out/r04v_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encoder']['ms'])")"
done
