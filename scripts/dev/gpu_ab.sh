set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
AB_PAIRS=${AB_PAIRS:-4} AB_STEPS=${AB_STEPS:-300} bash scripts/dev/ab_tree.sh run 2>&1 | tee gpurun_out/ab/ab_${AB_TAG:-x}.txt
