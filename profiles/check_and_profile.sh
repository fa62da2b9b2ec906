#!/bin/bash
# GPU box, repo root: the parity suites, then a rocprofv3 kernel trace of bench.py at config C and at config E.
#   bash profiles/check_and_profile.sh TAG [pytest files...]
# Writes gpurun_out/gputest_TAG.txt, gpurun_out/prof_TAG{,_E}/ and gpurun_out/bench_prof_TAG{,_E}.json; stops at the
# first failing step.
set -uo pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
TESTS=("$@")
[ ${#TESTS[@]} -eq 0 ] && TESTS=(tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_errors.py)
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread "${TESTS[@]}" > "$OUT/gputest_$TAG.txt" 2>&1
rc=$?
echo "tests $rc"
[ $rc -eq 0 ] || exit $rc
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$OUT/bench_prof_$TAG.json" 2>&1
rc=$?
echo "bench C $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_E" -o run -- \
    python3 "$R/bench.py" --config E --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > "$OUT/bench_prof_${TAG}_E.json" 2>&1
rc=$?
echo "bench E $rc"
exit $rc
