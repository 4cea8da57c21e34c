#!/bin/bash
# Round 4: rehearsal of bench.py's N > 1 control flow on one GPU (two ranks sharing it, gloo,
# eager): every post-timed-region probe must run its collectives on every rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TM_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --eager --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04x.log 2>&1
rc=$?
grep -v "^#" gpurun_out/r04x.log | tail -3 | cut -c1-400
exit $rc
