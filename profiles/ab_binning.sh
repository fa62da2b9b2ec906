#!/bin/bash
# Same-box A/B of the two binnings (GPU box, repo root): bench.py with the row binning and with OMR_BINNING=sort,
# alternating ROUNDS times, at the bench args given (e.g. --config E).  ROUNDS=2 bash profiles/ab_binning.sh [args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
ROUNDS=${ROUNDS:-2}
mkdir -p "$R/gpurun_out/abbin"
for ((r = 0; r < ROUNDS; r++)); do
    timeout -k 10 240 python3 "$R/bench.py" --no-cpu-baseline --no-train-step "$@" > "$R/gpurun_out/abbin/rows_$r.json" 2>/dev/null || exit 1
    OMR_BINNING=sort timeout -k 10 240 python3 "$R/bench.py" --no-cpu-baseline --no-train-step "$@" > "$R/gpurun_out/abbin/sort_$r.json" 2>/dev/null || exit 1
done
python3 - "$R/gpurun_out/abbin" "$ROUNDS" <<'PY'
import json, statistics, sys
d, n = sys.argv[1], int(sys.argv[2])
for name in ("rows", "sort"):
    runs = [json.loads([l for l in open(f"{d}/{name}_{r}.json") if l.startswith("{")][-1]) for r in range(n)]
    st = {k: round(statistics.median(x["stages_ms"][k] for x in runs), 4) for k in runs[0]["stages_ms"]}
    print(name, [round(x["value"], 1) for x in runs], [round(x["ms_per_step"], 4) for x in runs], st)
PY
