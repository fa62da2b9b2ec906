set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05g}
# the training step with the SH copy kept current by Adam (omr_adam_step_sh_out): tests, then its kernel trace
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_losses.py tests/test_gpu_train_dist.py tests/test_gpu_renderer.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_train" -o run -- \
    python3 "$R/profiles/train_prof.py" --config C --steps 10 > "$R/gpurun_out/${TAG}_train.json" 2> "$R/gpurun_out/${TAG}_train.err"
echo "train prof rc=$?"; cat "$R/gpurun_out/${TAG}_train.json"
cd $R
timeout -k 10 300 python3 profiles/train_prof.py --config C --steps 20 > gpurun_out/${TAG}_train_noprof.json 2>&1
echo "train rc=$?"; tail -1 gpurun_out/${TAG}_train_noprof.json
