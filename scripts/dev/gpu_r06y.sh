set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06y
mkdir -p $O
for lib in libtransmil_hip.so libtransmil_hip_noslp.so; do
  echo "== $lib"; TRANSMIL_HIP_LIB=transmil_deepgraft_amd/$lib timeout -k 10 120 python scripts/dev/a3_split_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee $O/a3_split_noslp.txt
echo "== env A/B: product (A) vs nystrom.hip without SLP vectorisation (B)"
AB_ENV_A="" AB_ENV_B="TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_noslp.so" AB_PAIRS=4 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_noslp.txt
