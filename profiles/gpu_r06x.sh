set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06x}
# equirect preprocess without the staged SH spans: per-lane rows in registers (lon_lane, 4 waves per SIMD) or the
# colour from the row in global memory (lon_global, 7 waves); the C parity case through lon_lane, then the
# interleaved A/B at C
OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp_lon/lon_lane.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "lonlat_1k or lonlat_ragged or baseline_config_full and C" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
EXP_DIR=$R/omnigs-fork_amd/lib/exp_lon ROUNDS=3 timeout -k 10 900 bash profiles/ab3.sh > gpurun_out/${TAG}_ab_C.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_C.txt
