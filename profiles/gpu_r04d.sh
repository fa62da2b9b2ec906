# config A / B kernel traces (launch overhead study) + parity of the default build
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "parity or generic or unaligned or scale_modifier" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04d_gputest.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04d_gputest.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp; export TMPDIR=/tmp
for c in A B; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r04d_$c -o run -- \
    python3 $R/bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-train-step > $R/gpurun_out/r04d_bench_$c.json 2> $R/gpurun_out/r04d_bench_$c.err
  rc=$?; echo "prof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 $R/profiles/gaps.py $R/gpurun_out/prof_r04d_$c --last-steps 10 > $R/gpurun_out/r04d_gaps_$c.txt 2>&1
  head -30 $R/gpurun_out/r04d_gaps_$c.txt
done
