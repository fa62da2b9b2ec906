set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05u}
# render kernel knobs at C: backward batch 32 / 48 (40 default), 7 waves per SIMD (batch 40 / 32), forward batch 48 / 32
for r in 0 1; do
  echo "== C round $r" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 500 bash profiles/ab.sh --config C --steps 20 --warmup 5 >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
done
cat gpurun_out/${TAG}_ab.txt
