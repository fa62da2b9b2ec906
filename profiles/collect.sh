#!/bin/bash
# Collect the round's profiles on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of bench.py          -> gpurun_out/prof_<tag>/ (bench.py's default 5 warm-up
#      and, with STEPS=20, its 20 timed steps: the launch times still fall over the first ~20 steps of a fresh
#      process, so the profile's timed window should be the bench's own; profiles/r05z_kernel_stats.csv)
#   2. rocprofv3 --pmc FETCH_SIZE (own pass)                  -> gpurun_out/pmc_fetch_<tag>/
#   3. rocprofv3 --pmc WRITE_SIZE (own pass)                  -> gpurun_out/pmc_write_<tag>/
# Counters are collected in their own runs with no trace domains besides the kernel trace
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass).
# profiles/pmc_summarize.py then turns the CSVs into profiles/<tag>_*.csv and profiles/pmc_latest.json.
set -euo pipefail
TAG=${1:?round tag, e.g. r01e}
STEPS=${2:-10}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup "${WARMUP:-5}" --no-cpu-baseline --no-train-step > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err"
echo "[collect] kernel trace done"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > "$OUT/bench_pmc_fetch_$TAG.json" 2> "$OUT/pmc_fetch_$TAG.err"
echo "[collect] FETCH_SIZE done"
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > "$OUT/bench_pmc_write_$TAG.json" 2> "$OUT/pmc_write_$TAG.err"
echo "[collect] WRITE_SIZE done"
