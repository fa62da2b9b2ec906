set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06r}
# small views: the row binning (default) against the emit + radix-sort binning (OMR_BINNING=sort)
for cfg in A B; do
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_$cfg timeout -k 10 600 bash profiles/ab_env.sh "rows" "sort:OMR_BINNING=sort" -- --config $cfg > gpurun_out/${TAG}_ab_$cfg.txt 2>&1
echo "ab $cfg rc=$?"; cat gpurun_out/${TAG}_ab_$cfg.txt
done
