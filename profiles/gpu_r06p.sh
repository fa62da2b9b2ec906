set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06p}
# small views, every workgroup resident: the forward without the longest-first tile order and the backward schedule
# without its sort. Parity with both forced off at every config (both backward mappings, one-wave forward), then the
# A/B at A and B: both skipped (the default there), the tile order back, the sort back, both back
OMR_FWD_TILE_ORDER=0 OMR_BWD_SCHED_SORT=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "test_parity or render_depth or baseline_config_full or backward_mappings or two_band or one_wave" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity_unordered.txt 2>&1
rc=$?; echo "parity unordered rc=$rc"; tail -1 gpurun_out/${TAG}_parity_unordered.txt; [ $rc -eq 0 ] || exit 1
for cfg in A B; do
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg timeout -k 10 600 bash profiles/ab_env.sh "auto" "order:OMR_FWD_TILE_ORDER=1" "sort:OMR_BWD_SCHED_SORT=1" "both:OMR_FWD_TILE_ORDER=1,OMR_BWD_SCHED_SORT=1" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_A_$TAG" -o run -- \
    python3 "$R/bench.py" --config A --steps 20 --warmup 5 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_A_prof_$TAG.json" 2> "$R/gpurun_out/bench_A_prof_$TAG.err"
echo "A kernel stats rc=$?"
