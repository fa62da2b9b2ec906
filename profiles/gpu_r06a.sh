set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06a}
# round 6, first run: smoke, the whole GPU suite (libm-oracle parity, split pinhole preprocess, RCCL one-rank
# exchange, Adam without the SH row walk), the pinhole preprocess A/B (split vs fused) at E pinhole, its kernel
# statistics, and the default bench line
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_Ep timeout -k 10 600 bash profiles/ab_env.sh "split" "fused:OMR_PRE_SPLIT=0" -- --config E_pinhole > gpurun_out/${TAG}_ab_Ep.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_Ep.txt
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_E_pinhole_$TAG" -o run -- \
    python3 "$R/bench.py" --config E_pinhole --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_E_pinhole_prof_$TAG.json" 2> "$R/gpurun_out/bench_E_pinhole_prof_$TAG.err"
echo "E_pinhole kernel stats rc=$?"
cd $R
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench C rc=$?"; head -c 300 gpurun_out/bench_C_$TAG.json
