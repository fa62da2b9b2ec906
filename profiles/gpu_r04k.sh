set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# side-stream SH colour: fork point (0 preprocess / 1 depth sort / 2 scans) x grid cap; parity of the default first
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04k_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04k_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=2 timeout -k 10 500 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04k_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04k_ab_C.txt
ROUNDS=2 timeout -k 10 700 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04k_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04k_ab_E.txt
