set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# timeout -k 10 300 python -u -m pytest tests/test_gpu_sh_jac.py tests/test_capi_host.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04t_shjac_test.txt 2>&1
# rc=$?; echo "sh_jac tests rc=$rc"; tail -3 gpurun_out/r04t_shjac_test.txt; [ $rc -eq 0 ] || exit 1
# backward_schedule_kernel loads in flight (unroll 4 / SG 8 default; 16; 32): kernel times from rocprofv3 at C and E
cd /tmp && export TMPDIR=/tmp
for b in base sched16 sched32; do
  lib=""; [ $b != base ] && lib=$R/omnigs-fork_amd/lib/exp/$b.so
  for cfg in C E; do
    OMR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04t_${b}_$cfg -o run -- \
        python3 $R/bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > $R/gpurun_out/r04t_${b}_$cfg.json 2> $R/gpurun_out/r04t_${b}_$cfg.err || exit 1
    grep -h backward_schedule $R/gpurun_out/r04t_${b}_$cfg/run_kernel_stats.csv | cut -d, -f2-5 | sed "s/^/$b $cfg /"
  done
done
