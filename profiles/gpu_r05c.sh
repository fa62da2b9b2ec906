set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-r05c}
# kernel traces of the depth sort variants (bits = depth_sort, bytes = OMR_DEPTH_SORT=bytes) at C and E
cd /tmp
export TMPDIR=/tmp
for cfg in C E; do
  for v in bits bytes; do
    if [ $v = bytes ]; then export OMR_DEPTH_SORT=bytes; else unset OMR_DEPTH_SORT; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_${cfg}_$v" -o run -- \
      python3 "$R/bench.py" --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-train-step > "$OUT/bench_prof_${TAG}_${cfg}_$v.json" 2> "$OUT/bench_prof_${TAG}_${cfg}_$v.err"
    echo "[$cfg $v] rc=$?"
  done
done
