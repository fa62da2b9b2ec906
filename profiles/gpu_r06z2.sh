set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06z2}
# forward scans bounded by the culled-aside depth sort's visible count (pinhole views): the parity file (every pinhole
# case, both depth-sort paths, both binnings) and the libm pinhole cases, then the interleaved A/B at E pinhole
# against every rank scanned (scan_all)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_libm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 900 bash profiles/ab3.sh --config E_pinhole > gpurun_out/${TAG}_ab_E_pinhole.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_E_pinhole.txt
