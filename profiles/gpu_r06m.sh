set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06m}
# the depth sort by counting, LDS-staged: parity subset, A/B at A, kernel statistics
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "depth_sort or count_sort or test_parity or baseline_config_full" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_A timeout -k 10 600 bash profiles/ab_env.sh "count" "radix:OMR_DEPTH_SORT=bytes" -- --config A > gpurun_out/${TAG}_ab_A.txt 2>&1
echo "ab A rc=$?"; cat gpurun_out/${TAG}_ab_A.txt
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_A_$TAG" -o run -- \
    python3 "$R/bench.py" --config A --steps 20 --warmup 5 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_A_prof_$TAG.json" 2> "$R/gpurun_out/bench_A_prof_$TAG.err"
echo "A kernel stats rc=$?"
grep -i "count_sort" "$R/gpurun_out/prof_A_$TAG/run_kernel_stats.csv"
