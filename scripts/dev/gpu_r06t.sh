set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_pinv_split_gpu.py tests/test_parity_gpu.py tests/test_bench_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
echo "== tree A/B: bf16 A3 backward dq~ slabs (A) vs HEAD (B)"
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_a3_bwd_bf16_slab.txt
