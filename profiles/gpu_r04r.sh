set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# sh_jac rows staged flat in LDS and stored as float4 (default) vs nine strided 4-B stores per lane (jacstrided)
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_renderer.py tests/test_gpu_libtorch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04r_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04r_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 300 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04r_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04r_ab_C.txt
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04r_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04r_ab_E.txt
