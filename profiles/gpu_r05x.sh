set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05x}
# wave_rows_store: every LDS read before the stores (no store waiting for the previous one through a reused register)
# vs HEAD (lib/exp/rows_store_old.so): gaussian_bwd dL_dsh rows, preprocess render records
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh_jac.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for r in 0 1; do
  for cfg in C E E_pinhole; do
    echo "== $cfg round $r" >> gpurun_out/${TAG}_ab.txt
    timeout -k 10 400 bash profiles/ab.sh --config $cfg --steps 20 --warmup 5 >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/${TAG}_ab.txt
