set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06y}
# C without the forward tile order (OMR_FWD_TILE_ORDER=0; at B it cost 6 us, C was never measured), interleaved A/B;
# then E pinhole kernel statistics of the tree with the LDS-free pinhole preprocess
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_C timeout -k 10 900 bash profiles/ab_env.sh "base" "noorder:OMR_FWD_TILE_ORDER=0" -- --config C > gpurun_out/${TAG}_ab_C.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_C.txt
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_E_pinhole_$TAG" -o run -- \
    python3 "$R/bench.py" --config E_pinhole --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_E_pinhole_prof_$TAG.json" 2> "$R/gpurun_out/bench_E_pinhole_prof_$TAG.err"
echo "E_pinhole kernel stats rc=$?"
