set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05v}
# diagnostic: preprocess without its SH row traffic (every row load reads one broadcast line; wrong colours) — what
# the rows cost the kernel at C and E
for cfg in C E; do
  echo "== $cfg" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 500 bash profiles/ab.sh --config $cfg --steps 20 --warmup 5 >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
done
cat gpurun_out/${TAG}_ab.txt
