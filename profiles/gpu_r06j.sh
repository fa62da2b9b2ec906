set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06j}
# render_fwd bands per wave at the small views: 1 (four waves per tile), 2 (default below 16 k tiles), 4
OMR_FWD_BANDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "test_parity or render_depth or baseline_config_full" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity_fwd1.txt 2>&1
rc=$?; echo "parity fwd1 rc=$rc"; tail -1 gpurun_out/${TAG}_parity_fwd1.txt; [ $rc -eq 0 ] || exit 1
for cfg in A B; do
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg timeout -k 10 600 bash profiles/ab_env.sh "two" "one:OMR_FWD_BANDS=1" "four:OMR_FWD_BANDS=4" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt
done
