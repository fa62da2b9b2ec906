set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# pinhole preprocess with the SH rows requested after the geometry, for the visible lanes only (late): parity, then an
# interleaved A/B at E pinhole (lonlat instantiations are unchanged)
OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/late.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh_jac.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04p3_gputest_late.txt 2>&1
rc=$?; echo "late parity rc=$rc"; tail -1 gpurun_out/r04p3_gputest_late.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 300 bash profiles/ab3.sh --config E_pinhole --steps 10 --warmup 3 > gpurun_out/r04p3_ab_Ep.txt 2>&1
echo "ab Ep rc=$?"; cat gpurun_out/r04p3_ab_Ep.txt
