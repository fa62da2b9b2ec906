set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05zy}
# after the pinhole span stores (b628583): smoke, the whole GPU suite, the bench lines, E pinhole and E kernel statistics
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench C rc=$?"
for cfg in E E_pinhole; do
    timeout -k 10 200 python3 bench.py --config "$cfg" --no-cpu-baseline > "gpurun_out/bench_${cfg}_$TAG.json" 2> "gpurun_out/bench_${cfg}_$TAG.err"
    echo "bench $cfg rc=$?"
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_E_pinhole_$TAG" -o run -- \
    python3 "$R/bench.py" --config E_pinhole --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_E_pinhole_prof_$TAG.json" 2> "$R/gpurun_out/bench_E_pinhole_prof_$TAG.err"
echo "E_pinhole kernel stats rc=$?"
