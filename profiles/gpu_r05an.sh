set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05an}
# gaussian_bwd at equirect views requesting the per-Gaussian inputs before radii (in-tree) vs after it (gbwd_old)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh_jac.py tests/test_gpu_exchange_overlap.py tests/test_gpu_parallel.py tests/test_gpu_libtorch.py tests/test_gpu_renderer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for r in 0 1; do
  echo "== E_pinhole round $r" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 400 bash profiles/ab.sh --config E_pinhole --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
  echo "== C round $r" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 400 bash profiles/ab.sh --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
done
echo "== E round 0" >> gpurun_out/${TAG}_ab.txt
timeout -k 10 400 bash profiles/ab.sh --config E --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_ab.txt
