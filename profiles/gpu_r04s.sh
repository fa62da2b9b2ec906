set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# gaussian_bwd_jac_kernel (no SH rows, half-image dL_dsh staging): GPU suite, then A/B against the one-image kernel
# (nogbjac) and the 5-wave build (jacw5, 4 VGPRs spilled)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04s_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04s_gputest.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 300 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04s_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04s_ab_C.txt
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04s_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04s_ab_E.txt
