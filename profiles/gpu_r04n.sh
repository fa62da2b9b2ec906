set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# render_bwd batch size sweep (base = 64)
ROUNDS=3 timeout -k 10 500 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04n_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04n_ab_C.txt
ROUNDS=2 timeout -k 10 500 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04n_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04n_ab_E.txt
ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config B --steps 30 --warmup 5 > gpurun_out/r04n_ab_B.txt 2>&1
echo "ab B rc=$?"; cat gpurun_out/r04n_ab_B.txt
