#!/bin/bash
# Config C5 at its own size on one GPU: scripts/bench_c5.py (4096 tiles -> ResNet-50 -> TransMIL(2048),
# train step) in eval-BN and train-BN encoder modes, then a rocprofv3 kernel trace of the eval run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
for mode in eval train; do
  timeout -k 10 400 python scripts/bench_c5.py --n 4096 --steps ${STEPS:-4} --warmup 2 --encoder-mode $mode \
    > gpurun_out/c5_${TAG}_$mode.log 2>&1 || { tail -20 gpurun_out/c5_${TAG}_$mode.log; exit 1; }
  tail -1 gpurun_out/c5_${TAG}_$mode.log | cut -c1-400
done
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_${TAG} -o run --output-format csv -- \
    python3 scripts/bench_c5.py --n 4096 --steps 2 --warmup 1 --encoder-mode eval > gpurun_out/c5prof_${TAG}.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/c5prof_${TAG}.log | cut -c1-200; exit $rc
fi
