set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# the SH colour on a side stream (OMR_PRE_SPLIT): the whole GPU suite, then A/B against the fused preprocess
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04j_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04j_gputest.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04j_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04j_ab_C.txt
ROUNDS=2 timeout -k 10 500 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04j_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04j_ab_E.txt
ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config A --steps 50 --warmup 10 > gpurun_out/r04j_ab_A.txt 2>&1
echo "ab A rc=$?"; cat gpurun_out/r04j_ab_A.txt
ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config B --steps 30 --warmup 5 > gpurun_out/r04j_ab_B.txt 2>&1
echo "ab B rc=$?"; cat gpurun_out/r04j_ab_B.txt
