set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05z2}
# the round-end profile of C again over exactly the bench's default window (5 warm-up, 20 timed steps; the launch
# times still fall over the first ~20 steps of a fresh process), then the bench line reading it
timeout -k 10 600 bash profiles/collect.sh $TAG 20
echo "collect rc=$?"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_C_$TAG.json 2> gpurun_out/bench_C_$TAG.err
echo "bench rc=$?"
