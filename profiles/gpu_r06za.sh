set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06za}
# render_fwd / render_bwd compiled with other LLVM machine-scheduler strategies (-mllvm -amdgpu-sched-strategy=
# max-ilp / iterative-ilp / max-memory-clause; same VGPR occupancy), interleaved A/B at C against the default
ROUNDS=3 timeout -k 10 1000 bash profiles/ab3.sh --config C > gpurun_out/${TAG}_ab_C.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_C.txt
