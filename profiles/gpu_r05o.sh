set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05o}
# (1) preprocess: SH rows transposed in two column groups (7 KiB LDS per wave), 4 waves per SIMD, vs HEAD's 13 KiB
#     image at 3 waves (lib/exp/pre_old.so);
# (2) columns scatter: chunk descriptors by scalar loads, write-out with a fixed count of buffer stores, vs HEAD's
#     bin.hip (lib/exp/bin_old.so);
# (3) render kernels: tile order / ranges / units by scalar loads, vs HEAD's (lib/exp/render_old.so)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh_jac.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for r in 0 1; do
  for cfg in C E; do
    echo "== $cfg round $r" >> gpurun_out/${TAG}_ab.txt
    timeout -k 10 500 bash profiles/ab.sh --config $cfg --steps 20 --warmup 5 >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
  done
done
echo "== E_pinhole round 0" >> gpurun_out/${TAG}_ab.txt
timeout -k 10 500 bash profiles/ab.sh --config E_pinhole --steps 20 --warmup 5 >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_ab.txt
