set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06zf}
# the final tree of round 6 (after the pinhole preprocess and scan changes): smoke, the whole GPU suite (parity residuals recorded), the default bench line,
# the LibTorch boundary, the other configurations, the training step at C
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench C rc=$?"
timeout -k 10 200 python3 bench.py --boundary libtorch --no-cpu-baseline > "gpurun_out/bench_lt_$TAG.json" 2> "gpurun_out/bench_lt_$TAG.err"
echo "libtorch rc=$?"
for cfg in A B E E_pinhole; do
timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > "gpurun_out/bench_${cfg}_$TAG.json" 2> "gpurun_out/bench_${cfg}_$TAG.err"
echo "bench $cfg rc=$?"
done
timeout -k 10 120 python3 profiles/train_prof.py --config C --steps 30 > gpurun_out/${TAG}_train_noprof.json 2> gpurun_out/${TAG}_train_noprof.err
echo "train rc=$?"; tail -c 400 gpurun_out/${TAG}_train_noprof.json
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for c in ("C", "lt", "A", "B", "E", "E_pinhole"):
    f = f"gpurun_out/bench_{c}_{t}.json"
    j = json.loads(open(f).read().strip().splitlines()[-1])
    r = j["roofline"]
    print(c, j["value"], j["ms_per_step"], r["kernel"], r["frac"], r.get("frac_rocprof"), r.get("valu_issue_frac"))
PY
cd /tmp
export TMPDIR=/tmp
for cfg in E E_pinhole; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${cfg}_$TAG" -o run -- \
    python3 "$R/bench.py" --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > "$R/gpurun_out/bench_${cfg}_prof_$TAG.json" 2> "$R/gpurun_out/bench_${cfg}_prof_$TAG.err"
echo "$cfg kernel stats rc=$?"
done
