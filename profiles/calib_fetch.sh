#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration per access pattern (GPU box, repo root): bash profiles/calib_fetch.sh
# Build first (CPU side): hipcc --offload-arch=gfx950 -O3 -o profiles/_build/calib_fetch profiles/calib_fetch.hip
# Then: python profiles/calib_summarize.py  -> profiles/<tag>_calib.json
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- "$R/profiles/_build/calib_fetch" > "$OUT/calib_known.json"
echo "[calib] FETCH_SIZE done"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o run -- "$R/profiles/_build/calib_fetch" > /dev/null
echo "[calib] WRITE_SIZE done"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/calib_trace" -o run -- "$R/profiles/_build/calib_fetch" > /dev/null
echo "[calib] trace done"
