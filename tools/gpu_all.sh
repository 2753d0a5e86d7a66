# every GPU test + smoke (what the driver runs at round end)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/full_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/full_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; exit $rc
