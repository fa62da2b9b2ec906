set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06k}
# columns-pass chunk of the row binning at the small views: 2048 slots (default below 2^25 instances), 1024, 512
for sh in 9 10; do
OMR_BIN_COLS_SHIFT=$sh timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary_checks.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity_cs$sh.txt 2>&1
rc=$?; echo "parity cols shift $sh rc=$rc"; tail -1 gpurun_out/${TAG}_parity_cs$sh.txt; [ $rc -eq 0 ] || exit 1
done
for cfg in A B C; do
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg timeout -k 10 600 bash profiles/ab_env.sh "2048" "1024:OMR_BIN_COLS_SHIFT=10" "512:OMR_BIN_COLS_SHIFT=9" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt
done
