set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
# SQ counters of the render probes / packed pairs at C and of the ranks at E (OR tables vs ballots)
for b in base fwd_valu4 bwd_valu4 fwd_pairs bwd_pairs; do
  lib=""; [ $b != base ] && lib=$R/omnigs-fork_amd/lib/sq/$b.so
  OMR_LIB_PATH=$lib timeout -k 10 400 bash profiles/sq.sh r04g_$b --no-train-step || exit 1
  echo "sq $b done"
done
for b in base rank_ballot; do
  lib=""; [ $b != base ] && lib=$R/omnigs-fork_amd/lib/sq/$b.so
  OMR_LIB_PATH=$lib timeout -k 10 400 bash profiles/sq.sh r04gE_$b --config E --no-train-step || exit 1
  echo "sq E $b done"
done
