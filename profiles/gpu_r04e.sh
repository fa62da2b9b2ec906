set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
ROUNDS=3 timeout -k 10 600 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04e_ab.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/r04e_ab.txt
