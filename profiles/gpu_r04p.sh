set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# row_valid zeroed by render_fwd (OMR_RV_FWD) instead of the columns scatter: full GPU suite, then A/B (rvold)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04p_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04p_gputest.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 300 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04p_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04p_ab_C.txt
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04p_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04p_ab_E.txt
ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config A --steps 50 --warmup 10 > gpurun_out/r04p_ab_A.txt 2>&1
echo "ab A rc=$?"; cat gpurun_out/r04p_ab_A.txt
