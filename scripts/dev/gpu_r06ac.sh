set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ac
mkdir -p $O
timeout -k 10 200 python scripts/dev/dxn_splitk.py 2>&1 | grep -v amdgpu.ids | tee $O/dxn_splitk.txt
