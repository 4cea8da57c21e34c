set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ao
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
echo "== tree A/B: step_prepare cast with 8 pieces per lane (A) vs 4 (HEAD, B)"
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_cast_pieces8.txt
