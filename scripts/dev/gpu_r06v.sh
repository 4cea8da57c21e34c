set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 700 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_bench_gpu.py tests/test_siblings_gpu.py tests/test_ddp_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
echo "== tree A/B: bf16 conv dv (A) vs HEAD (B)"
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_conv_dv_bf16.txt
