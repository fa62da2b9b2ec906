set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06f}
# render_bwd with two waves per unit / two bands per wave (OMR_BWD_BANDS=2, paired and unpaired reductions):
# parity first, then an interleaved A/B at C and E and SQ passes of both mappings at C
for v in "2 1" "2 0"; do
  set -- $v
  OMR_BWD_BANDS=$1 OMR_BWD2_PAIR=$2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "test_parity or baseline_config_full or long_and_huge or white or one_wave" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity_b$1p$2.txt 2>&1
  rc=$?; echo "parity bands=$1 pair=$2 rc=$rc"; tail -1 gpurun_out/${TAG}_parity_b$1p$2.txt; [ $rc -eq 0 ] || exit 1
done
ROUNDS=3 AB_OUT=$R/gpurun_out/${TAG}_ab_C timeout -k 10 900 bash profiles/ab_env.sh "base" "b2:OMR_BWD_BANDS=2" "b2u:OMR_BWD_BANDS=2,OMR_BWD2_PAIR=0" -- --config C > gpurun_out/${TAG}_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/${TAG}_ab_C.txt
ROUNDS=1 AB_OUT=$R/gpurun_out/${TAG}_ab_E timeout -k 10 600 bash profiles/ab_env.sh "base" "b2:OMR_BWD_BANDS=2" "b2u:OMR_BWD_BANDS=2,OMR_BWD2_PAIR=0" -- --config E > gpurun_out/${TAG}_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/${TAG}_ab_E.txt
OMR_BWD_BANDS=2 timeout -k 10 400 bash profiles/sq.sh ${TAG}_b2 --no-train-step
echo "sq b2 rc=$?"
OMR_BWD_BANDS=2 OMR_BWD2_PAIR=0 timeout -k 10 400 bash profiles/sq.sh ${TAG}_b2u --no-train-step
echo "sq b2u rc=$?"
