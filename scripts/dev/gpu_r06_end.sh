set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_final.sh || exit 1
bash scripts/dev/gpu_r06q.sh
