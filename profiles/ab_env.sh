#!/bin/bash
# Interleaved A/B of run-time switches (GPU box, repo root): one build, variants given as NAME or NAME:VAR=VAL,VAR=VAL
# (NAME alone = the default). ROUNDS rounds alternate the variants so slow drifts of the box's clock hit all alike.
# Prints per variant the median MP/s, ms/step and per-stage ms (bench.py's per-stage pass).
#   ROUNDS=2 bash profiles/ab_env.sh "base" "bytes:OMR_DEPTH_SORT=bytes" -- --config C
R=${GRAFT_REPO_ROOT:-$(pwd)}
ROUNDS=${ROUNDS:-2}
OUT=${AB_OUT:-$R/gpurun_out/ab_env}
variants=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do variants+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
rm -rf "$OUT"
mkdir -p "$OUT"
for ((r = 0; r < ROUNDS; r++)); do
    for v in "${variants[@]}"; do
        name=${v%%:*}
        envs=""
        [ "$v" != "$name" ] && envs=${v#*:}
        env ${envs//,/ } timeout -k 10 240 python3 "$R/bench.py" --no-cpu-baseline --no-train-step "$@" \
            > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit 1
    done
done
python3 - "$OUT" "${variants[@]}" <<'PY'
import json, statistics, sys
d = sys.argv[1]
for v in sys.argv[2:]:
    name = v.split(":")[0]
    runs = []
    for r in range(100):
        try:
            runs.append(json.loads(open(f"{d}/{name}_{r}.json").read().strip().splitlines()[-1]))
        except (OSError, IndexError):
            break
    med = statistics.median(x["value"] for x in runs)
    ms = statistics.median(x["ms_per_step"] for x in runs)
    st = {k: round(statistics.median(x["stages_ms"][k] for x in runs), 4) for k in runs[0]["stages_ms"]}
    print(name, round(med, 1), round(ms, 4), [round(x["value"], 1) for x in runs], st)
PY
