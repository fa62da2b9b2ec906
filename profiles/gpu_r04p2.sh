set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# the pruned tree: smoke + GPU suite; the SH rows gathered through a half-column image in preprocess (halves, 4 waves
# per SIMD; halves_w5: 5 waves, 23 VGPRs spilled): parity of halves, then interleaved A/B at C, E pinhole and E
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04p2_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r04p2_smoke.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04p2_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/r04p2_gputest.txt; [ $rc -eq 0 ] || exit 1
OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/halves.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh_jac.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04p2_gputest_halves.txt 2>&1
rc=$?; echo "halves parity rc=$rc"; tail -1 gpurun_out/r04p2_gputest_halves.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 300 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04p2_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04p2_ab_C.txt
ROUNDS=3 timeout -k 10 300 bash profiles/ab3.sh --config E_pinhole --steps 10 --warmup 3 > gpurun_out/r04p2_ab_Ep.txt 2>&1
echo "ab Ep rc=$?"; cat gpurun_out/r04p2_ab_Ep.txt
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04p2_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04p2_ab_E.txt
timeout -k 10 60 omnigs-fork_amd/lib/test/write_bw 1.5 > gpurun_out/r04p2_write_bw.txt 2>&1
echo "write_bw rc=$?"; cat gpurun_out/r04p2_write_bw.txt
