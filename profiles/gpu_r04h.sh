set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# the default build (rows info fused, OR-table ranks): the whole GPU suite, residuals recorded
OMR_PARITY_RESIDUALS=$R/gpurun_out/r04h_residuals.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04h_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04h_gputest.txt; [ $rc -eq 0 ] || exit 1
# A/B against the ballot ranks (rank_ballot) and the separate rows-info launch (info_sep)
ROUNDS=2 timeout -k 10 500 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04h_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04h_ab_C.txt
ROUNDS=2 timeout -k 10 600 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04h_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04h_ab_E.txt
ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config A --steps 50 --warmup 10 > gpurun_out/r04h_ab_A.txt 2>&1
echo "ab A rc=$?"; cat gpurun_out/r04h_ab_A.txt
# a smaller backward segment (CKPT) for the small views: more units per long tile
EXP_DIR=$R/omnigs-fork_amd/lib/exp_ck ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config A --steps 50 --warmup 10 > gpurun_out/r04h_ck_A.txt 2>&1
echo "ck A rc=$?"; cat gpurun_out/r04h_ck_A.txt
EXP_DIR=$R/omnigs-fork_amd/lib/exp_ck ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config B --steps 30 --warmup 5 > gpurun_out/r04h_ck_B.txt 2>&1
echo "ck B rc=$?"; cat gpurun_out/r04h_ck_B.txt
EXP_DIR=$R/omnigs-fork_amd/lib/exp_ck ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04h_ck_C.txt 2>&1
echo "ck C rc=$?"; cat gpurun_out/r04h_ck_C.txt
