#!/bin/bash
# A/B the default build against variants in omnigs-fork_amd/lib/exp/*.so (GPU box, from the repo root):
#   bash profiles/ab.sh [bench args...]  -> one line per build: name, MP/s, per-stage ms
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
run() {
    local name=$1 lib=$2
    shift 2
    OMR_LIB_PATH=$lib timeout -k 10 240 python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/ab_$name.json" 2> "$R/gpurun_out/ab_$name.err" || return 1
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/ab_$name.json')); print('$name', d['value'], d['stages_ms'])"
}
run base "" "$@" || exit 1
for so in "$R"/omnigs-fork_amd/lib/exp/*.so; do
    [ -e "$so" ] || continue
    run "$(basename "$so" .so)" "$so" "$@" || exit 1
done
