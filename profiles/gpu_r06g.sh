set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06g}
# the committed tree: smoke, the whole GPU suite (parity residuals recorded), the default bench line (reads
# profiles/pmc_latest.json: roofline.valu_issue_frac), the LibTorch boundary
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench C rc=$?"
timeout -k 10 200 python3 bench.py --boundary libtorch --no-cpu-baseline > "gpurun_out/bench_lt_$TAG.json" 2> "gpurun_out/bench_lt_$TAG.err"
echo "libtorch rc=$?"
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/bench_C_{t}.json", f"gpurun_out/bench_lt_{t}.json"):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    r = j["roofline"]
    print(f, j["value"], j["ms_per_step"], r["kernel"], r["frac"], r.get("frac_rocprof"), r.get("valu_issue_frac"))
PY
