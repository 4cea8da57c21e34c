set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06f
mkdir -p $O
make -C transmil_deepgraft_amd/csrc diag -j16 > $O/make_diag.txt 2>&1 || { tail -5 $O/make_diag.txt; exit 1; }
export TRANSMIL_HIP_LIB=$PWD/transmil_deepgraft_amd/libtransmil_hip_diag.so
timeout -k 10 200 python -u scripts/microbench.py --gemm-ab --only gemm > $O/gemm_ab.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/microbench.py --gemm-ab --only wgrad > $O/wgrad_ab.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/dev/gemm_stamps2.py > $O/gemm_stamps2.txt 2>&1 || exit 1
cat $O/gemm_ab.txt $O/wgrad_ab.txt
