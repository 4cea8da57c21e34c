set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 120 python -u scripts/dev/a3_split_time.py > $O/a3_split.txt 2>&1 || { cat $O/a3_split.txt; exit 1; }
cat $O/a3_split.txt
make -C transmil_deepgraft_amd/csrc diag -j16 > $O/make_diag.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/dev/a3_fwd_stamps.py > $O/a3_fwd_stamps_nosim2.txt 2>&1 || exit 1
tail -6 $O/a3_fwd_stamps_nosim2.txt
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "a1_bwd_dqkv" > $O/tests.txt 2>&1; rc=$?; tail -3 $O/tests.txt; exit $rc
