#!/bin/bash
# Round-end refresh on the GPU box (repo root, via gpurun): profiles of config C (profiles/collect.sh), the bench line
# of every BASELINE config, the LibTorch boundary, and config E's kernel statistics. Summarise on the CPU side with
#   python3 profiles/pmc_summarize.py TAG   (and copy gpurun_out/bench_*_TAG.json into profiles/)
set -euo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
bash "$R/profiles/collect.sh" "$TAG" 10
cd "$R"
timeout -k 10 300 python3 bench.py > "$OUT/bench_C_$TAG.json" 2> "$OUT/bench_C_$TAG.err"
echo "[refresh] C done"
for cfg in A B E E_pinhole; do
    timeout -k 10 200 python3 bench.py --config "$cfg" --no-cpu-baseline > "$OUT/bench_${cfg}_$TAG.json" 2> "$OUT/bench_${cfg}_$TAG.err"
    echo "[refresh] $cfg done"
done
timeout -k 10 200 python3 bench.py --boundary libtorch --no-cpu-baseline > "$OUT/bench_lt_$TAG.json" 2> "$OUT/bench_lt_$TAG.err"
echo "[refresh] libtorch done"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_E_$TAG" -o run -- \
    python3 "$R/bench.py" --config E --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$OUT/bench_E_prof_$TAG.json" 2> "$OUT/bench_E_prof_$TAG.err"
echo "[refresh] E kernel stats done"
