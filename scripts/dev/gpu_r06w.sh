set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06w
mkdir -p $O
echo "== env A/B: wgrad slots default (A) vs 512 (B)"
AB_ENV_A="" AB_ENV_B="TM_WGRAD_SLOTS=512" AB_PAIRS=3 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_wgrad_slots512.txt || exit 1
echo "== env A/B: LN bwd rpb 8 (A) vs 16 (B)"
AB_ENV_A="" AB_ENV_B="TM_LN_BWD_RPB=16" AB_PAIRS=3 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_ln_rpb16.txt || exit 1
echo "== env A/B: LN bwd rpb 8 (A) vs 4 (B)"
AB_ENV_A="" AB_ENV_B="TM_LN_BWD_RPB=4" AB_PAIRS=3 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_ln_rpb4.txt
