set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05m}
# SSIM strip height A/B (lib/exp/ssim_r*.so) on the prefetching streaming kernel
for r in 0 1 2; do
  for so in base omnigs-fork_amd/lib/exp/ssim_r*.so; do
    name=$(basename $so .so)
    if [ $name = base ]; then unset OMR_LIB_PATH; else export OMR_LIB_PATH=$R/$so; fi
    echo "$name $(timeout -k 10 120 python3 profiles/bench_loss.py 2>/dev/null | tail -1)" >> gpurun_out/${TAG}_ssim_ab.txt
  done
done
unset OMR_LIB_PATH
cat gpurun_out/${TAG}_ssim_ab.txt
