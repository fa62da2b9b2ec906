set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# default: render_bwd batch 40 for views with more units than resident slots, 64 below; parity first
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_renderer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04o_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04o_parity.txt; [ $rc -eq 0 ] || exit 1
# A/B: b64 (64 everywhere), b28w7 (28 + 7 waves/SIMD, spills), fb32 / fb48 (forward batches)
ROUNDS=3 timeout -k 10 500 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04o_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04o_ab_C.txt
ROUNDS=2 timeout -k 10 500 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04o_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04o_ab_E.txt
ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config B --steps 30 --warmup 5 > gpurun_out/r04o_ab_B.txt 2>&1
echo "ab B rc=$?"; cat gpurun_out/r04o_ab_B.txt
