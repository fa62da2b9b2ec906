set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06b}
# counters of the split pinhole preprocess (geometry + colour kernels) at E pinhole: SQ passes and FETCH / WRITE
timeout -k 10 400 bash profiles/sq.sh ${TAG}_Ep --config E_pinhole --no-train-step
echo "sq rc=$?"
cd /tmp
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_${c}_${TAG}_Ep" -o run -- \
    python3 "$R/bench.py" --config E_pinhole --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > "$R/gpurun_out/pmc_${c}_${TAG}_Ep.json" 2> "$R/gpurun_out/pmc_${c}_${TAG}_Ep.err"
echo "$c rc=$?"
done
cd $R
ROUNDS=2 AB_OUT=$R/gpurun_out/${TAG}_ab_Ep timeout -k 10 600 bash profiles/ab_env.sh "split" "fused:OMR_PRE_SPLIT=0" -- --config E_pinhole > gpurun_out/${TAG}_ab_Ep.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_Ep.txt
