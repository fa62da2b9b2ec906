set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# render_bwd staging batch 48 / 56 against 40 (LDS 6656 / 7040 B per one-wave workgroup against 6272): parity of 48,
# then interleaved A/B at C and E
OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/bwd48.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04p4_gputest_bwd48.txt 2>&1
rc=$?; echo "bwd48 parity rc=$rc"; tail -1 gpurun_out/r04p4_gputest_bwd48.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 300 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04p4_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04p4_ab_C.txt
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04p4_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04p4_ab_E.txt
