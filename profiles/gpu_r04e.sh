set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for v in fwd_pairs bwd_pairs sched; do
  OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/$v.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_baseline_config_full[C]" tests/test_gpu_parity.py -k "test_parity or two_wave or one_wave or baseline_config_full" --deselect "tests/test_gpu_parity.py::test_baseline_config_full[B]" --deselect "tests/test_gpu_parity.py::test_baseline_config_full[E]" --deselect "tests/test_gpu_parity.py::test_baseline_config_full[E_pinhole]" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04e_gputest_$v.txt 2>&1
  echo "tests $v rc=$?"; tail -2 gpurun_out/r04e_gputest_$v.txt
done
ROUNDS=2 timeout -k 10 700 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04e_ab.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/r04e_ab.txt
# config E: the backward schedule over 8 x K blocks (sched.so) vs base, 2 rounds interleaved
mkdir -p gpurun_out/abE
for r in 0 1; do
  for b in base sched; do
    lib=""; [ $b = sched ] && lib=$R/omnigs-fork_amd/lib/exp/sched.so
    OMR_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config E --steps 10 --warmup 3 --no-cpu-baseline --no-train-step > gpurun_out/abE/${b}_$r.json 2> gpurun_out/abE/${b}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], {k: round(v,4) for k,v in d['stages_ms'].items()})" gpurun_out/abE/${b}_$r.json $b
  done
done
