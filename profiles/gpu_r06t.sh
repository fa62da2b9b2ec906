set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06t}
# pinhole preprocess with per-lane SH row loads (no 13-KiB LDS image: 4 waves per SIMD instead of 3): the pinhole
# parity cases (oracle and libm oracle), then the interleaved A/B at E pinhole against the staged spans (pre_span)
# and a 5-waves-per-SIMD build (pre_w5)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_libm.py -m gpu -k "pinhole or E_pinhole" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 900 bash profiles/ab3.sh --config E_pinhole > gpurun_out/${TAG}_ab_E_pinhole.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_E_pinhole.txt
