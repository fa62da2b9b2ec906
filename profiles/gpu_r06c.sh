set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06c}
# the pinhole colour kernel's variants: cooperative row gather or per-lane rows, mask words per wave; split vs fused
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "split or outside_the_predicted or E_pinhole" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_split_tests.txt 2>&1
rc=$?; echo "split tests rc=$rc"; tail -2 gpurun_out/${TAG}_split_tests.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=2 AB_OUT=$R/gpurun_out/${TAG}_ab_Ep timeout -k 10 900 bash profiles/ab_env.sh "coop" "lane:OMR_COLOUR_COOP=0" "fused:OMR_PRE_SPLIT=0" -- --config E_pinhole > gpurun_out/${TAG}_ab_Ep.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_Ep.txt
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_E_pinhole_$TAG" -o run -- \
    python3 "$R/bench.py" --config E_pinhole --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_E_pinhole_prof_$TAG.json" 2> "$R/gpurun_out/bench_E_pinhole_prof_$TAG.err"
echo "E_pinhole kernel stats rc=$?"
grep -h preprocess "$R"/gpurun_out/prof_E_pinhole_$TAG/*kernel_stats.csv | cut -c1-200
