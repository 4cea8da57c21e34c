set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06w
mkdir -p $O
echo "== env A/B: wgrad slots default (A) vs 512 (B)"
AB_ENV_A="" AB_ENV_B="TM_WGRAD_SLOTS=512" AB_PAIRS=3 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_wgrad_slots512.txt || exit 1
echo "== env A/B: LN bwd rpb 8 (A) vs 16 (B)"
AB_ENV_A="" AB_ENV_B="TM_LN_BWD_RPB=16" AB_PAIRS=3 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_ln_rpb16.txt || exit 1
echo "== env A/B: LN bwd rpb 8 (A) vs 4 (B)"
AB_ENV_A="" AB_ENV_B="TM_LN_BWD_RPB=4" AB_PAIRS=3 bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_ln_rpb4.txt || exit 1
echo "== tests + tree A/B: bf16 PPEG weight-gradient slabs (A) vs HEAD (B)"
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_kernels_gpu.py -k "ppeg or transmil or bf16_mode or c2" > $O/tests_ppeg.txt 2>&1
rc=$?; tail -2 $O/tests_ppeg.txt; [ $rc -eq 0 ] || exit $rc
AB_PAIRS=3 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_ppeg_bf16_slab.txt
