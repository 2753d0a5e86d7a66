# LocalInertialBA / LBA parity + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lia.py tests/test_gpu_lba.py > gpurun_out/lia_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lia_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_lba.py --lia --calls 20 --cpu-calls 1 2>/dev/null | tail -c 400 || exit 1
timeout -k 10 200 python tools/bench_lba.py --lia --large --calls 10 --cpu-calls 1 2>/dev/null | tail -c 400 || exit 1
