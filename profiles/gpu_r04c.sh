set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "parity or generic or unaligned or scale_modifier or config_full and C" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04c_gputest.txt 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r04c_gputest.txt
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 600 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04c_ab.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/r04c_ab.txt
