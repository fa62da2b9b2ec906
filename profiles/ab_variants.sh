#!/bin/bash
# Kernel-time A/B of library variants (GPU box, repo root): for each NAME, a rocprofv3 kernel trace of bench.py with
# OMR_LIB_PATH=omnigs-fork_amd/lib/exp/NAME.so (build_variant.sh), then the average duration of the kernels matching
# KERNELS (a regex).   KERNELS='rows_scatter|cols_scatter' bash profiles/ab_variants.sh "--config E" NAME...
R=${GRAFT_REPO_ROOT:-$(pwd)}
ARGS=${1:?bench args}
shift
OUT=$R/gpurun_out/abvar
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for n in "$@"; do
    OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/$n.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/$n" -o run -- python3 "$R/bench.py" $ARGS --steps 3 --warmup 1 --no-cpu-baseline --no-train-step \
        > "$OUT/$n.json" 2>&1 || exit 1
done
python3 - "$OUT" "${KERNELS:-scatter}" "$@" <<'PY'
import csv, glob, json, re, sys
d, pat, names = sys.argv[1], sys.argv[2], sys.argv[3:]
for n in names:
    f = glob.glob(f"{d}/{n}/**/*kernel_stats.csv", recursive=True)[0]
    ks = {}
    for r in csv.DictReader(open(f)):
        if re.search(pat, r["Name"]):
            m = re.search(r"(\w+_kernel)(<\d+)?", r["Name"])
            ks[m.group(1) + (m.group(2) or "")] = float(r["AverageNs"]) / 1e3
    b = json.loads([l for l in open(f"{d}/{n}.json") if l.startswith("{")][-1])
    print(n, round(b["ms_per_step"], 4), {k: round(v, 1) for k, v in sorted(ks.items())})
PY
