#!/bin/bash
# Round 4: C5 conv1x1 hipBLASLt candidates timed once per shape (tiles per encoder piece), eval and train BN, MIOpen find on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_encoder.py > gpurun_out/r04w_t.log 2>&1 || { tail -30 gpurun_out/r04w_t.log; exit 1; }
tail -1 gpurun_out/r04w_t.log
for cfg in "eval 1024" "train 1024"; do
  set -- $cfg
  timeout -k 10 400 python -u scripts/bench_c5.py --encoder-mode $1 --chunk $2 --steps 3 --warmup 2 \
    > gpurun_out/r04w_$1_$2.log 2>&1 || { tail -20 gpurun_out/r04w_$1_$2.log; exit 1; }
  echo "$1 $2 $(tail -1 gpurun_out/r04w_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encoder']['ms'])")"
done
