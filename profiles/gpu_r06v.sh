set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r06v}
# pinhole gaussian_bwd with per-lane dL_dsh rows and masked span zeros (OMR_GBWD_PIN_LANE=1, the in-tree build): the
# pinhole / skip_dsh / sh_jac / boundary tests, then the interleaved A/B at E pinhole against the staged image
# (gb_span) and a 4-waves-per-SIMD build (gb_lane4)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_libm.py tests/test_gpu_sh_jac.py tests/test_gpu_boundary_checks.py -m gpu -k "pinhole or skip_dsh or sh_jac or stored or sh_row or boundary or E_pinhole" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/${TAG}_parity.txt; [ $rc -eq 0 ] || exit 1
ROUNDS=3 timeout -k 10 900 bash profiles/ab3.sh --config E_pinhole > gpurun_out/${TAG}_ab_E_pinhole.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/${TAG}_ab_E_pinhole.txt
