set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05ac}
# columns scatter: in-tree (next chunk staged before the write-out, 1024 staged owners) vs HEAD (cols_old) vs HEAD with
# 1024 staged owners (old_own1024); then per-phase stamps of the old and new kernels at E
for r in 0 1; do
  echo "== E round $r" >> gpurun_out/${TAG}_ab.txt
  timeout -k 10 400 bash profiles/ab.sh --config E --steps 20 --warmup 5 --no-train-step >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
done
for v in old new; do
  OMR_LIB_PATH=omnigs-fork_amd/lib/stamps/${v}_stamps.so timeout -k 10 200 python3 profiles/bin_stamps.py E > gpurun_out/${TAG}_stamps_$v.json 2>gpurun_out/${TAG}_stamps_$v.err || exit 1
done
cat gpurun_out/${TAG}_ab.txt gpurun_out/${TAG}_stamps_*.json
