set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06q}
# forward scans without the end-of-chain gathers: parity (every parity test), then A / B / C against the build
# before it (omnigs-fork_amd/lib/exp/prev.so, build_variant.sh from the previous commit's sources)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
for cfg in A B C; do
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg timeout -k 10 600 bash profiles/ab_env.sh "new" "prev:OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/prev.so" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt
done
