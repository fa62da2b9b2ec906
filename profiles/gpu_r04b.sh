set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export OMR_PARITY_RESIDUALS=$R/gpurun_out/r04b_residuals.jsonl
rm -f $OMR_PARITY_RESIDUALS
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b_gputest.txt 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r04b_gputest.txt
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 600 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04b_ab.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/r04b_ab.txt
