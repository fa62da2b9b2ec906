set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05d}
# render_bwd latency levers: interleaved A/B of lib/exp/*.so against the default build at C, with
# the timed loop's live render_bwd launch time, then SQ counters of every build
ROUNDS=3 timeout -k 10 900 bash profiles/ab3.sh > gpurun_out/${TAG}_ab_C.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_C.txt | cut -c1-300
python3 profiles/ab_live.py gpurun_out/ab3 > gpurun_out/${TAG}_ab_live.txt; cat gpurun_out/${TAG}_ab_live.txt
for so in base omnigs-fork_amd/lib/exp/*.so; do
  name=$(basename $so .so)
  if [ $name = base ]; then unset OMR_LIB_PATH; else export OMR_LIB_PATH=$R/$so; fi
  timeout -k 10 400 bash profiles/sq.sh ${TAG}_$name --no-train-step > /dev/null 2>&1
  echo "sq $name rc=$?"
done
unset OMR_LIB_PATH
cd /tmp
export TMPDIR=/tmp
for v in bits bytes; do
  if [ $v = bytes ]; then export OMR_DEPTH_SORT=bytes; else unset OMR_DEPTH_SORT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_C_$v" -o run -- \
    python3 "$R/bench.py" --config C --steps 10 --warmup 3 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_prof_${TAG}_C_$v.json" 2> "$R/gpurun_out/bench_prof_${TAG}_C_$v.err"
  echo "[prof C $v] rc=$?"
done
