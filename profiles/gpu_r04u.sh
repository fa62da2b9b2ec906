set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# backward_schedule_kernel with register-resident shares: parity + renderer tests, then kernel times (rocprofv3) and A/B
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_renderer.py tests/test_gpu_sh_jac.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04u_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04u_parity.txt; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
for b in base schedold; do
  lib=""; [ $b != base ] && lib=$R/omnigs-fork_amd/lib/exp/$b.so
  for cfg in C E; do
    OMR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04u_${b}_$cfg -o run -- \
        python3 $R/bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > $R/gpurun_out/r04u_${b}_$cfg.json 2> $R/gpurun_out/r04u_${b}_$cfg.err || exit 1
    echo "$b $cfg done"
  done
done
cd $R
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04u_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04u_ab_E.txt
