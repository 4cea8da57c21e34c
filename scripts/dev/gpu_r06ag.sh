set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm" tests/test_parity_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
make -C transmil_deepgraft_amd/csrc diag -j16 > $O/diag_build.txt 2>&1 || exit 1
TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so timeout -k 10 200 python scripts/dev/qkv_big_stamps.py 2>&1 | grep -v amdgpu.ids | tee $O/qkv_big_stamps.txt
echo "== tree A/B: 128-row passes + incremental (bag, t) in the QKV epilogue (A) vs HEAD (B)"
AB_PAIRS=4 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_big_epi128_inc.txt
