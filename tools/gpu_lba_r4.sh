# Round 4: LBA / LIA parity + timing (+ the back-end rocprof evidence with PROF=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lia.py > gpurun_out/lba_r4_tests.log 2>&1; rc=$?; tail -8 gpurun_out/lba_r4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_lba.py --calls 20 --cpu-calls 1 > gpurun_out/bench_lba.json 2>/dev/null || exit 1
tail -c 600 gpurun_out/bench_lba.json; echo
timeout -k 10 200 python tools/bench_lba.py --lia --calls 20 --cpu-calls 1 > gpurun_out/bench_lia.json 2>/dev/null || exit 1
tail -c 600 gpurun_out/bench_lia.json; echo
if [ "${PROF:-0}" = 1 ]; then ROUND=r04 bash tools/ba_prof.sh > gpurun_out/ba_prof.log 2>&1; rc=$?; tail -30 gpurun_out/ba_prof.log; exit $rc; fi
