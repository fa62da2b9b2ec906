set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r05q}
# Adam's f_dc + f_rest blocks issue every load before their barrier (one round trip) vs HEAD (lib/exp/adam_prev.so)
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gputest.txt; [ $rc -eq 0 ] || exit 1
for r in 0 1 2; do
  for so in base omnigs-fork_amd/lib/exp/adam_prev.so; do
    name=$(basename $so .so)
    if [ $name = base ]; then unset OMR_LIB_PATH; else export OMR_LIB_PATH=$R/$so; fi
    echo "$name $(BENCH_OPTIM_HIP_ONLY=1 timeout -k 10 120 python3 profiles/bench_optim.py 2>/dev/null | tail -1)" >> gpurun_out/${TAG}_adam_ab.txt
  done
done
unset OMR_LIB_PATH
cat gpurun_out/${TAG}_adam_ab.txt
for r in 0 1 2; do timeout -k 10 120 python3 profiles/train_prof.py --config C --steps 30 >> gpurun_out/${TAG}_train_noprof.json; done
cat gpurun_out/${TAG}_train_noprof.json
