# Round 4 final call A: the whole GPU suite, smoke, back-end profiles (r04)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/final_tests.log 2>&1; rc=$?; tail -3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -2 gpurun_out/final_smoke.log
ROUND=r04 bash tools/ba_prof.sh > gpurun_out/final_ba.log 2>&1 || { tail -5 gpurun_out/final_ba.log; exit 1; }
grep -v "^ " gpurun_out/final_ba.log | tail -4
