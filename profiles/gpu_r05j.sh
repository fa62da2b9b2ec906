set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05j}
# the SSIM streaming kernel with 11-row register prefetch, fused + packed taps: tests, A/B vs the previous kernel
# (lib/exp/ssim_old.so), train-step trace
timeout -k 10 600 python -u -m pytest tests/test_gpu_losses.py tests/test_gpu_train_dist.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for r in 0 1 2; do
  for so in base omnigs-fork_amd/lib/exp/ssim_old.so; do
    name=$(basename $so .so)
    if [ $name = base ]; then unset OMR_LIB_PATH; else export OMR_LIB_PATH=$R/$so; fi
    echo "$name $(timeout -k 10 120 python3 profiles/bench_loss.py 2>/dev/null | tail -1)" >> gpurun_out/${TAG}_ssim_ab.txt
    echo "$name 4k $(timeout -k 10 120 python3 profiles/bench_loss.py 2048 4096 2>/dev/null | tail -1)" >> gpurun_out/${TAG}_ssim_ab.txt
  done
done
unset OMR_LIB_PATH
cat gpurun_out/${TAG}_ssim_ab.txt
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_train" -o run -- \
    python3 "$R/profiles/train_prof.py" --config C --steps 10 > "$R/gpurun_out/${TAG}_train.json" 2> "$R/gpurun_out/${TAG}_train.err"
echo "train prof rc=$?"; cat "$R/gpurun_out/${TAG}_train.json"
