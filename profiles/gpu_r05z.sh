set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05z}
# end-of-round check: smoke, the whole GPU suite (parity residuals recorded), SQ counters of C, the refresh (profiles
# of C with timed-window stats, every bench line, LibTorch, E kernel statistics), the training step
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit 1
OMR_PARITY_RESIDUALS=$R/gpurun_out/${TAG}_residuals.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 bash profiles/sq.sh $TAG --no-train-step
echo "sq rc=$?"
timeout -k 10 900 bash profiles/refresh.sh $TAG
echo "refresh rc=$?"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_train" -o run -- \
    python3 "$R/profiles/train_prof.py" --config C --steps 10 > "$R/gpurun_out/${TAG}_train.json" 2> "$R/gpurun_out/${TAG}_train.err"
echo "train prof rc=$?"
cd $R
timeout -k 10 120 python3 profiles/train_prof.py --config C --steps 30 > gpurun_out/${TAG}_train_noprof.json
echo "train rc=$?"; cat gpurun_out/${TAG}_train_noprof.json
