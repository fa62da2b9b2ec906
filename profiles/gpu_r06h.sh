set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06h}
# the two-bands-per-wave render_bwd at the small views (A, B), where every unit is resident at once
for cfg in B A; do
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg timeout -k 10 600 bash profiles/ab_env.sh "base" "b2:OMR_BWD_BANDS=2" "b2u:OMR_BWD_BANDS=2,OMR_BWD2_PAIR=0" "b2_64:OMR_BWD_BANDS=2,OMR_BWD2_BATCH=64" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt
done
