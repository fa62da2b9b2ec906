set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05a}
# round 5, first box: smoke, the whole GPU suite (new boundary / sh_jac / 8-rank overlapped exchange tests), the
# round's first profiles of config C (kernel trace -> timed-window stats, FETCH / WRITE passes) and the bench line
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=15 > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 600 bash profiles/collect.sh $TAG 10
echo "collect rc=$?"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench rc=$?"; cat gpurun_out/bench_C_$TAG.json | head -c 600
