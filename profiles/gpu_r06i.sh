set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06i}
# small views take the two-waves-per-unit render backward by default: the parity suite, then A / B / C bench lines
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_renderer.py tests/test_gpu_libtorch.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_A timeout -k 10 600 bash profiles/ab_env.sh "auto" "four:OMR_BWD_BANDS=4" -- --config A > gpurun_out/${TAG}_ab_A.txt 2>&1
echo "ab A rc=$?"; cat gpurun_out/${TAG}_ab_A.txt
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_B timeout -k 10 600 bash profiles/ab_env.sh "auto" "four:OMR_BWD_BANDS=4" -- --config B > gpurun_out/${TAG}_ab_B.txt 2>&1
echo "ab B rc=$?"; cat gpurun_out/${TAG}_ab_B.txt
ROUNDS=2 AB_OUT=$R/gpurun_out/${TAG}_ab_C timeout -k 10 600 bash profiles/ab_env.sh "auto" "four:OMR_BWD_BANDS=4" -- --config C > gpurun_out/${TAG}_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/${TAG}_ab_C.txt
