set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05b}
# depth sort over the varying bits: parity (new depth-sort cases, every config at full size), then the A/B against
# the 4 x 8-bit sort (OMR_DEPTH_SORT=bytes) at C, E, E pinhole and A
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh_jac.py tests/test_gpu_boundary_checks.py -x -v --timeout 300 --timeout-method thread --durations=10 > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for cfg in C E E_pinhole A; do
    AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg ROUNDS=2 timeout -k 10 600 bash profiles/ab_env.sh "bits" "bytes:OMR_DEPTH_SORT=bytes" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
    echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt | cut -c1-400
done
