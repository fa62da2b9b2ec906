set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04m_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r04m_smoke.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 1200 bash profiles/refresh.sh r04m
echo "refresh rc=$?"
# render_bwd batch size (LDS per wave: 64 -> 7424 B, 48 -> 6656 B, 40 -> 6272 B)
ROUNDS=3 timeout -k 10 400 bash profiles/ab3.sh --steps 20 --warmup 5 > gpurun_out/r04m_ab_C.txt 2>&1
echo "ab C rc=$?"; cat gpurun_out/r04m_ab_C.txt
ROUNDS=2 timeout -k 10 400 bash profiles/ab3.sh --config E --steps 10 --warmup 3 > gpurun_out/r04m_ab_E.txt 2>&1
echo "ab E rc=$?"; cat gpurun_out/r04m_ab_E.txt
