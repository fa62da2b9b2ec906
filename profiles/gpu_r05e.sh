set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05e}
# depth sort: onesweep passes 1..3 take nvis from their digit totals (no count word); parity of the depth-sort cases,
# A/B at C, A, E pinhole; then a kernel trace of the training step at C
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "depth_sort or baseline_config_full or parity" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for cfg in C A E_pinhole; do
    AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg ROUNDS=3 timeout -k 10 600 bash profiles/ab_env.sh "bits" "bytes:OMR_DEPTH_SORT=bytes" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
    echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt | cut -c1-300
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_train" -o run -- \
    python3 "$R/profiles/train_prof.py" --config C --steps 10 > "$R/gpurun_out/${TAG}_train.json" 2> "$R/gpurun_out/${TAG}_train.err"
echo "train prof rc=$?"; cat "$R/gpurun_out/${TAG}_train.json"
