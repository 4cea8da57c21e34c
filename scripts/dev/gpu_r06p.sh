set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06p
mkdir -p $O
L=transmil_deepgraft_amd
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_interface.py tests/test_bench_gpu.py tests/test_siblings_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for lib in ab/$L/libtransmil_hip.so $L/libtransmil_hip_o512.so $L/libtransmil_hip.so $L/libtransmil_hip_o2048.so; do
  TRANSMIL_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-hbm-probe 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], 'opt_ms', d.get('optimizer_ms'))" || exit 1
done | tee $O/opt_variants.txt
echo "== tree A/B: grid-stride optimizer (A) vs HEAD (B)"
AB_PAIRS=3 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_opt.txt
