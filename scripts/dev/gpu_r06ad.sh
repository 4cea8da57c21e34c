set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ad
mkdir -p $O
timeout -k 10 300 python scripts/dev/gemm_vs_blaslt.py 2>&1 | grep -v amdgpu.ids | tee $O/gemm_vs_blaslt.txt
