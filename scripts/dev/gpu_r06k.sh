set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 200 python -u scripts/dev/wgrad_splits.py > $O/wgrad_splits.txt 2>&1; rc=$?; cat $O/wgrad_splits.txt; exit $rc
