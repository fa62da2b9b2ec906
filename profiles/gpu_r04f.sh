set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# the default build (row info fused into the rows scatter): the whole GPU suite, residuals recorded
OMR_PARITY_RESIDUALS=$R/gpurun_out/r04f_residuals.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04f_gputest.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04f_gputest.txt; [ $rc -eq 0 ] || exit 1
OMR_LIB_PATH=$R/omnigs-fork_amd/lib/exp/fwd_tsub.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_baseline_config_full[C]" tests/test_gpu_parity.py -k "test_parity or two_wave or one_wave" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04f_gputest_fwd_tsub.txt 2>&1
rc=$?; echo "tests fwd_tsub rc=$rc"; tail -2 gpurun_out/r04f_gputest_fwd_tsub.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=2 timeout -k 10 500 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04f_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04f_ab_C.txt
ROUNDS=2 timeout -k 10 600 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04f_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04f_ab_E.txt
# render_bwd WRITE_SIZE with and without the row_valid marks (bwd_nomark: diagnostic, wrong gradients)
cd /tmp && export TMPDIR=/tmp
for b in base bwd_nomark; do
  lib=""; [ $b = bwd_nomark ] && lib=$R/omnigs-fork_amd/lib/exp/bwd_nomark.so
  OMR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r04f_write_$b -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > $R/gpurun_out/r04f_write_$b.json 2> $R/gpurun_out/r04f_write_$b.err || exit 1
  echo "write pass $b done"
done
