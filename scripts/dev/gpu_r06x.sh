set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06x
mkdir -p $O
echo "== env A/B: LN bwd rpb 8 (A) vs 16 (B)"
AB_ENV_A="" AB_ENV_B="TM_LN_BWD_RPB=16" AB_PAIRS=5 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_ln_rpb16.txt || exit 1
echo "== env A/B: LN bwd rpb 8 (A) vs 32 (B)"
AB_ENV_A="" AB_ENV_B="TM_LN_BWD_RPB=32" AB_PAIRS=4 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_ln_rpb32.txt
