# Full validation of the current build: GPU tests, smoke, inertial latency, default bench.
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python tools/bench_latency_inertial.py --frames 100 > gpurun_out/lat_inertial.json 2>gpurun_out/lat_inertial.err || exit 1
tail -1 gpurun_out/lat_inertial.json
timeout -k 10 600 python bench.py > gpurun_out/bench_val.json 2>gpurun_out/bench_val.err || exit 1
tail -1 gpurun_out/bench_val.json
