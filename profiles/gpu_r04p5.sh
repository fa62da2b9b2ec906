set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
# HBM traffic of config E pinhole's kernels (gaussian_bwd: 88 % culled rows written as zeros), one counter pass each
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_r04p5" -o run -- \
    python3 "$R/bench.py" --config E_pinhole --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > "$OUT/r04p5_fetch.json" 2> "$OUT/r04p5_fetch.err"
echo "fetch rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_r04p5" -o run -- \
    python3 "$R/bench.py" --config E_pinhole --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > "$OUT/r04p5_write.json" 2> "$OUT/r04p5_write.err"
echo "write rc=$?"
