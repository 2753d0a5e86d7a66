set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/full_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/full_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_latency.py --frames 40 2>/dev/null | tail -c 700 || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/latprof -o lat -- python3 tools/lat_probe.py > gpurun_out/latprobe.log 2>&1 || exit 1
cat gpurun_out/latprobe.log
