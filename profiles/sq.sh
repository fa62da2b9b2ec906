#!/bin/bash
# SQ counter passes for the render kernels (GPU box, repo root): bash profiles/sq.sh TAG [bench args]
# Two --pmc passes (8 SQ slots each), kernel trace only; summarise with profiles/sq_summarize.py TAG.
set -euo pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d "$OUT/sq1_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$OUT/sq1_$TAG.json" 2> "$OUT/sq1_$TAG.err"
echo "[sq] pass 1 done"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVES \
    SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq2_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$OUT/sq2_$TAG.json" 2> "$OUT/sq2_$TAG.err"
echo "[sq] pass 2 done"
