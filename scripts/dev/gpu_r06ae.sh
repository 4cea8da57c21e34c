set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ae
mkdir -p $O
make -C transmil_deepgraft_amd/csrc diag -j16 > $O/diag_build.txt 2>&1 || exit 1
TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so timeout -k 10 200 python scripts/dev/qkv_big_stamps.py 2>&1 | grep -v amdgpu.ids | tee $O/qkv_big_stamps.txt
