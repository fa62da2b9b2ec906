set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05aq}
# render_bwd's point-list entries requested one batch ahead (in-tree) vs per batch (bwd_old)
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_renderer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for r in 0 1 2; do
  echo "== C round $r" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 400 bash profiles/ab.sh --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
done
for c in E B; do
echo "== $c round 0" >> gpurun_out/${TAG}_ab.txt
timeout -k 10 400 bash profiles/ab.sh --config $c --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
done
cat gpurun_out/${TAG}_ab.txt
