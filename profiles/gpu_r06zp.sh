set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06zz}
# the final tree of round 6, part 2: config C SQ passes (VALU-issue roofline), kernel trace over the bench window and
# FETCH / WRITE passes; E and E-pinhole kernel statistics
timeout -k 10 400 bash profiles/sq.sh $TAG --no-train-step
echo "sq rc=$?"
timeout -k 10 900 bash profiles/collect.sh $TAG 20
echo "collect rc=$?"
cd /tmp
export TMPDIR=/tmp
for cfg in E E_pinhole; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${cfg}_$TAG" -o run -- \
    python3 "$R/bench.py" --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_${cfg}_prof_$TAG.json" 2> "$R/gpurun_out/bench_${cfg}_prof_$TAG.err"
echo "$cfg kernel stats rc=$?"
done
