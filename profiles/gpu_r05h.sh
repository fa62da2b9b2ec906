set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05h}
# pinhole: compacted gaussian_bwd + onesweep passes 1..3 of the depth sort; the whole GPU suite, then A/Bs
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=12 > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
AB_OUT=$R/gpurun_out/${TAG}_ab_Ep ROUNDS=2 timeout -k 10 600 bash profiles/ab_env.sh "compact" "wave:OMR_GBWD_COMPACT=0" "plainsort:OMR_DEPTH_SORT=bytes" -- --config E_pinhole > gpurun_out/${TAG}_ab_Ep.txt 2>&1
echo "ab Ep rc=$?"; cut -c1-420 gpurun_out/${TAG}_ab_Ep.txt
AB_OUT=$R/gpurun_out/${TAG}_ab_C ROUNDS=1 timeout -k 10 300 bash profiles/ab_env.sh "base" -- --config C > gpurun_out/${TAG}_ab_C.txt 2>&1
echo "ab C rc=$?"; cut -c1-420 gpurun_out/${TAG}_ab_C.txt
