set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 120 python -u scripts/dev/a3_split_time.py > $O/a3_split.txt 2>&1 || { cat $O/a3_split.txt; exit 1; }
cat $O/a3_split.txt
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_pinv_split_gpu.py -k "sim2 or a3 or pinv or bf16 or parity or fixture or oracle" > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
AB_PAIRS=3 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_sim2_wave.txt
