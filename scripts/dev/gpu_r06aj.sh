set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06aj
mkdir -p $O
TM_RED_LOG=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-probe > $O/entries.txt 2>&1 || exit 1
grep "reduce entry" $O/entries.txt | sort | uniq -c | sort -rn | head -40
echo "== A: cap 262144, <= 12 splits per lane; B: default (65536, 24)"
AB_PAIRS=4 AB_ENV_A="TM_RED_CAP=262144 TM_RED_SPL=12" AB_ENV_B="" bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_red_v1.txt || exit 1
echo "== A: cap 1048576, <= 6 splits per lane; B: default"
AB_PAIRS=4 AB_ENV_A="TM_RED_CAP=1048576 TM_RED_SPL=6" AB_ENV_B="" bash scripts/dev/ab_env.sh 2>&1 | tee $O/ab_red_v2.txt
