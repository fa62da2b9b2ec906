set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05i}
# after r05h's fault (compacted gaussian_bwd wrote a NULL dL_dsh row under skip_dsh; fixed): the new pinhole paths'
# tests alone first, then the whole suite, then the A/Bs
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "compacted or depth_sort" -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_newpaths.txt 2>&1
rc=$?; echo "new paths rc=$rc"; tail -2 gpurun_out/${TAG}_newpaths.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=12 > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
AB_OUT=$R/gpurun_out/${TAG}_ab_Ep ROUNDS=2 timeout -k 10 600 bash profiles/ab_env.sh "compact" "wave:OMR_GBWD_COMPACT=0" "plainsort:OMR_DEPTH_SORT=bytes" -- --config E_pinhole > gpurun_out/${TAG}_ab_Ep.txt 2>&1
echo "ab Ep rc=$?"; cut -c1-420 gpurun_out/${TAG}_ab_Ep.txt
