set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06g
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm" > gpurun_out/r06g/tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r06g/tests.txt; [ $rc -eq 0 ] || exit $rc
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee gpurun_out/r06g/ab_bigtile_qkv.txt
