set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06aq
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "ppeg" tests/test_parity_gpu.py tests/test_reentrant_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
echo "== tree A/B: one-launch PPEG backward with weight-gradient and stencil blocks interleaved 1:3 (A) vs HEAD (B)"
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_ppeg_interleave.txt
