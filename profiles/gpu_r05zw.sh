set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05zw}
# after the render_bwd prologue change: smoke, the whole GPU suite, C's profiles over the bench window and the bench
# lines that read them (C, LibTorch)
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash profiles/collect.sh $TAG 20
echo "collect rc=$?"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench C rc=$?"
timeout -k 10 200 python3 bench.py --boundary libtorch --no-cpu-baseline > "gpurun_out/bench_lt_$TAG.json" 2> "gpurun_out/bench_lt_$TAG.err"
echo "libtorch rc=$?"
for cfg in E B; do
    timeout -k 10 200 python3 bench.py --config "$cfg" --no-cpu-baseline > "gpurun_out/bench_${cfg}_$TAG.json" 2> "gpurun_out/bench_${cfg}_$TAG.err"
    echo "bench $cfg rc=$?"
done
