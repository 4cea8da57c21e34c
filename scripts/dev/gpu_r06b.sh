set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06b
make -C transmil_deepgraft_amd/csrc diag -j16 > gpurun_out/r06b/make_diag.txt 2>&1 || { tail -5 gpurun_out/r06b/make_diag.txt; exit 1; }
timeout -k 10 200 python -u scripts/dev/pinv_graph_stamps.py --ab 0,6,0,6 --variant 6 > gpurun_out/r06b/pinv_stamps_wt.txt 2>&1
rc=$?; grep "A/B\|graph replay\|sum of" gpurun_out/r06b/pinv_stamps_wt.txt; exit $rc
