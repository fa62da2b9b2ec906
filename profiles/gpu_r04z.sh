set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r04z}
# end-of-round refresh: smoke, the whole GPU suite, then profiles/refresh.sh (kernel stats + PMC of C, every config's
# bench line, the LibTorch boundary, E kernel stats) and SQ counters of C
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 1000 bash profiles/refresh.sh $TAG
rc=$?; echo "refresh rc=$rc"; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 bash profiles/sq.sh $TAG --no-train-step
echo "sq rc=$?"
