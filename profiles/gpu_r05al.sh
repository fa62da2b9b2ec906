set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05al}
# gaussian_bwd over the visible list at pinhole views (two launches; the zero pass with span stores; in-tree) vs the wave kernel (gbwd_old)
timeout -k 10 900 python -u -m pytest tests/test_gpu_visible_list.py tests/test_gpu_parity.py tests/test_gpu_sh_jac.py tests/test_gpu_config_D_ranks.py tests/test_gpu_renderer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for r in 0 1 2; do
  echo "== E_pinhole round $r" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 400 bash profiles/ab.sh --config E_pinhole --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
done
echo "== C round 0" >> gpurun_out/${TAG}_ab.txt
timeout -k 10 400 bash profiles/ab.sh --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_ab.txt
