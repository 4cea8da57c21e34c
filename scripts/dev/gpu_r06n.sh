set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06n
mkdir -p $O
make -C transmil_deepgraft_amd/csrc diag -j16 > $O/diag_build.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/dev/a3_fwd_stamps.py > $O/a3_stamps_plain.txt 2>&1 || exit 1
A3_SIM2=1 timeout -k 10 120 python scripts/dev/a3_fwd_stamps.py > $O/a3_stamps_sim2.txt 2>&1 || exit 1
cat $O/a3_stamps_plain.txt $O/a3_stamps_sim2.txt
