mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/lba_quick.err
set -o pipefail
timeout -k 5 60 ./build/lba_solve_bench 18 200 || exit 1
timeout -k 5 60 ./build/lba_solve_bench 25 200 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lia.py > gpurun_out/lba_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lba_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_lba.py --calls 20 --cpu-calls 0 2>>gpurun_out/lba_quick.err | tail -c 250 || exit 1
timeout -k 10 200 python tools/bench_lba.py --lia --calls 20 --cpu-calls 0 2>>gpurun_out/lba_quick.err | tail -c 250 || exit 1
