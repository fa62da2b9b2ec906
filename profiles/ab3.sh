#!/bin/bash
# Interleaved A/B (GPU box, repo root): the default build and every lib/exp/*.so, ROUNDS rounds alternating, so slow
# drifts of the box's clock hit all builds alike. Prints per build the median MP/s and per-stage ms.
#   ROUNDS=3 bash profiles/ab3.sh [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
ROUNDS=${ROUNDS:-3}
rm -rf "$R/gpurun_out/ab3"
mkdir -p "$R/gpurun_out/ab3"
builds=("base:")
for so in "${EXP_DIR:-$R/omnigs-fork_amd/lib/exp}"/*.so; do
    [ -e "$so" ] && builds+=("$(basename "$so" .so):$so")
done
for ((r = 0; r < ROUNDS; r++)); do
    for b in "${builds[@]}"; do
        name=${b%%:*}
        lib=${b#*:}
        OMR_LIB_PATH=$lib timeout -k 10 240 python3 "$R/bench.py" --no-cpu-baseline --no-train-step "$@" \
            > "$R/gpurun_out/ab3/${name}_$r.json" 2> "$R/gpurun_out/ab3/${name}_$r.err" || exit 1
    done
done
python3 - "$R/gpurun_out/ab3" "${builds[@]}" <<'PY'
import json, statistics, sys
d = sys.argv[1]
for b in sys.argv[2:]:
    name = b.split(":")[0]
    runs = []
    for r in range(100):
        try:
            runs.append(json.load(open(f"{d}/{name}_{r}.json")))
        except OSError:
            break
    med = statistics.median(x["value"] for x in runs)
    st = {k: round(statistics.median(x["stages_ms"][k] for x in runs), 4) for k in runs[0]["stages_ms"]}
    print(name, round(med, 1), [round(x["value"], 1) for x in runs], st)
PY
