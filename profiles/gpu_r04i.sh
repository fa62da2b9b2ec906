set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# A/B: the depth sort's ranks by ballots (sort_ballot), backward segments of 512 (ck512)
ROUNDS=2 timeout -k 10 400 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04i_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04i_ab_C.txt
ROUNDS=2 timeout -k 10 500 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04i_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04i_ab_E.txt
ROUNDS=2 timeout -k 10 300 bash profiles/ab3.sh --config A --steps 50 --warmup 10 > gpurun_out/r04i_ab_A.txt 2>&1
echo "ab A rc=$?"; cat gpurun_out/r04i_ab_A.txt
# the columns scatter's phases at E with the OR-table ranks
OMR_LIB_PATH=$R/omnigs-fork_amd/lib/diag/binstamps.so timeout -k 10 200 python3 profiles/bin_stamps.py E > gpurun_out/r04i_bin_stamps_E.txt 2>&1
echo "stamps rc=$?"; cat gpurun_out/r04i_bin_stamps_E.txt
# SQ counters at C of the default build and of the packed band-pair variants
for b in base fwd_pairs bwd_pairs; do
  lib=""; [ $b != base ] && lib=$R/omnigs-fork_amd/lib/sq/$b.so
  OMR_LIB_PATH=$lib timeout -k 10 400 bash profiles/sq.sh r04i_$b --no-train-step || exit 1
  echo "sq $b done"
done
# render_bwd WRITE_SIZE with and without the row_valid marks (bwd_nomark: diagnostic, wrong gradients)
cd /tmp && export TMPDIR=/tmp
for b in base bwd_nomark; do
  lib=""; [ $b = bwd_nomark ] && lib=$R/omnigs-fork_amd/lib/diag/bwd_nomark.so
  OMR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r04i_write_$b -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-train-step > $R/gpurun_out/r04i_write_$b.json 2> $R/gpurun_out/r04i_write_$b.err || exit 1
  echo "write pass $b done"
done
