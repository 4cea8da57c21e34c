set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/dev/bench_configs.sh || exit 1
mkdir -p gpurun_out/r06q
for mode in eval train; do
  timeout -k 10 400 python scripts/bench_c5.py --n 4096 --steps 20 --warmup 2 --encoder-mode $mode \
    > gpurun_out/r06q/c5_$mode.log 2>&1 || { tail -20 gpurun_out/r06q/c5_$mode.log; exit 1; }
  tail -1 gpurun_out/r06q/c5_$mode.log | cut -c1-300
done
