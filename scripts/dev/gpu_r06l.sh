set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_interface.py tests/test_kernels_gpu.py tests/test_bench_gpu.py tests/test_siblings_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
echo "== env A/B: QKV big tile (A) vs ring (B)"
AB_ENV_A="" AB_ENV_B="TM_GEMM_QKV_BIG=0" AB_PAIRS=4 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_qkv_big_env.txt || exit 1
echo "== tree A/B: bf16 pre (A) vs HEAD (B)"
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_pre_bf16.txt
