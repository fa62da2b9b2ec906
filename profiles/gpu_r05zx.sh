set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05zx}
# round-end check of the final tree: smoke, the whole GPU suite (parity residuals recorded), SQ counters of C, C's
# profiles over the bench's own window (5 warm-up, 20 timed steps) and the bench line reading them, every other bench
# line, LibTorch, E kernel statistics, the training step
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 bash profiles/sq.sh $TAG --no-train-step
echo "sq rc=$?"
timeout -k 10 600 bash profiles/collect.sh $TAG 20
echo "collect rc=$?"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench C rc=$?"
for cfg in A B E E_pinhole; do
    timeout -k 10 200 python3 bench.py --config "$cfg" --no-cpu-baseline > "gpurun_out/bench_${cfg}_$TAG.json" 2> "gpurun_out/bench_${cfg}_$TAG.err"
    echo "bench $cfg rc=$?"
done
timeout -k 10 200 python3 bench.py --boundary libtorch --no-cpu-baseline > "gpurun_out/bench_lt_$TAG.json" 2> "gpurun_out/bench_lt_$TAG.err"
echo "libtorch rc=$?"
cd /tmp
export TMPDIR=/tmp
for cfg in E E_pinhole; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${cfg}_$TAG" -o run -- \
    python3 "$R/bench.py" --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_${cfg}_prof_$TAG.json" 2> "$R/gpurun_out/bench_${cfg}_prof_$TAG.err"
echo "$cfg kernel stats rc=$?"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_train" -o run -- \
    python3 "$R/profiles/train_prof.py" --config C --steps 10 > "$R/gpurun_out/${TAG}_train.json" 2> "$R/gpurun_out/${TAG}_train.err"
echo "train prof rc=$?"
cd $R
timeout -k 10 120 python3 profiles/train_prof.py --config C --steps 30 > gpurun_out/${TAG}_train_noprof.json
echo "train rc=$?"; cat gpurun_out/${TAG}_train_noprof.json
