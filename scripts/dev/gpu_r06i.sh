set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06i
mkdir -p $O
make -C transmil_deepgraft_amd/csrc diag -j16 > $O/make_diag.txt 2>&1 || exit 1
A3_SIM2=1 timeout -k 10 120 python -u scripts/dev/a3_fwd_stamps.py > $O/a3_fwd_stamps_sim2.txt 2>&1 || exit 1
tail -8 $O/a3_fwd_stamps_sim2.txt


