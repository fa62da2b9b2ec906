set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06w}
# pinhole preprocess evaluating the colour from the SH row in global memory (no 48 registers for it: 68 VGPRs, 7 waves
# per SIMD; pin_global8: 8 waves): the pinhole parity cases through the variant (ctypes path, OMR_LIB_PATH), then the
# interleaved A/B at E pinhole against the in-tree build (rows in registers, 4 waves per SIMD)
OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/pin_global.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_libm.py -m gpu -k "pinhole or E_pinhole" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 900 bash profiles/ab3.sh --config E_pinhole > gpurun_out/${TAG}_ab_E_pinhole.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_E_pinhole.txt
