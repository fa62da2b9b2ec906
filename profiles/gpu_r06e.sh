set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06e}
# config C: SQ counters (VALU issue roofline) and the kernel trace + FETCH / WRITE passes over the bench window
timeout -k 10 400 bash profiles/sq.sh $TAG --no-train-step
echo "sq rc=$?"
timeout -k 10 900 bash profiles/collect.sh $TAG 20
echo "collect rc=$?"
