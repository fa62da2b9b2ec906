set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export OMR_PARITY_RESIDUALS=$R/gpurun_out/r04a_residuals.jsonl
rm -f $OMR_PARITY_RESIDUALS
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04a_gputest.txt 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/r04a_gputest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err
echo "bench rc=$?"
tail -c 600 gpurun_out/r04a_bench.json
