set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06d
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee gpurun_out/r06d/ab_wt_all.txt || exit 1
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_pinv_split_gpu.py > gpurun_out/r06d/tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r06d/tests.txt; exit $rc
