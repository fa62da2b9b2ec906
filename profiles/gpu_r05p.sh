set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05p}
# densification statistics as extra blocks of the Adam launch: optimizer / training tests, train-step trace
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train_dist.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_train" -o run -- \
    python3 "$R/profiles/train_prof.py" --config C --steps 10 > "$R/gpurun_out/${TAG}_train.json" 2> "$R/gpurun_out/${TAG}_train.err"
echo "train prof rc=$?"
cd $R
for r in 0 1 2; do timeout -k 10 120 python3 profiles/train_prof.py --config C --steps 30 >> gpurun_out/${TAG}_train_noprof.json; done
cat gpurun_out/${TAG}_train_noprof.json
