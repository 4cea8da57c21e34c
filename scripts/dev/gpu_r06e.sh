set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06e
mkdir -p $O
make -C transmil_deepgraft_amd/csrc diag -j16 > $O/make_diag.txt 2>&1 || { tail -5 $O/make_diag.txt; exit 1; }
A3_SIM2=1 timeout -k 10 120 python -u scripts/dev/a3_fwd_stamps.py > $O/a3_fwd_stamps.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/dev/a1_bwd_stamps.py > $O/a1_bwd_stamps.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/dev/a3_bwd_stamps.py > $O/a3_bwd_stamps.txt 2>&1 || exit 1
tail -20 $O/a3_fwd_stamps.txt
