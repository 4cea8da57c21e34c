set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ak
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm" tests/test_parity_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
echo "== tree A/B: GEMM epilogue stores write-through (A) vs HEAD (B)"
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_gemm_epi_wt.txt
