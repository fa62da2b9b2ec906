set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06u}
# render_fwd: an instance reaching both bands of a two-band wave evaluated in one basic block (OMR_FWD_PAIR=1, the
# fwd_pair build in lib/exp2), interleaved A/B at C and B (two-band forward views)
for cfg in C B; do
EXP_DIR=$R/omnigs-fork_amd/lib/exp2 ROUNDS=3 timeout -k 10 900 bash profiles/ab3.sh --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
rc=$?; echo "ab $cfg rc=$rc"; cat gpurun_out/${TAG}_ab_$cfg.txt; [ $rc -eq 0 ] || exit 1
done
