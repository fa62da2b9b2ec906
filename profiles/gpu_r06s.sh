set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06s}
# small views take the emit + tile sort binning (at most 1024 tiles): the parity file (both binnings on the small
# cases), then the A/B at A against the row binning forced
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_A timeout -k 10 600 bash profiles/ab_env.sh "auto" "rows:OMR_BINNING=rows" -- --config A > gpurun_out/${TAG}_ab_A.txt 2>&1
echo "ab A rc=$?"; cat gpurun_out/${TAG}_ab_A.txt
