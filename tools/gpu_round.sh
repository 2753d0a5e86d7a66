#!/bin/bash
# One gpurun call: the LBA solve stamps, the LBA/LIA and extractor GPU tests,
# and the LBA/LIA timing lines.  Output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 ./build/lba_solve_bench 18 200 || exit 1
timeout -k 5 60 ./build/lba_solve_bench 25 200 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_lba.py tests/test_gpu_lia.py tests/test_gpu_extractor.py} > gpurun_out/round_tests.log 2>&1; rc=$?; tail -3 gpurun_out/round_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_lba.py --calls 20 --cpu-calls 0 2>/dev/null | tail -c 250 || exit 1
timeout -k 10 200 python tools/bench_lba.py --lia --calls 20 --cpu-calls 0 2>/dev/null | tail -c 250 || exit 1
if [ -n "${INERTIAL:-}" ]; then
  timeout -k 10 300 python tools/bench_inertial.py --problems 64 --calls 20 2>/dev/null | tail -c 600 || exit 1
fi
if [ -n "${LATINERT:-}" ]; then
  timeout -k 10 300 python tools/bench_latency_inertial.py --frames 16 2>gpurun_out/latinert.err | tail -c 1200 || { tail -5 gpurun_out/latinert.err; exit 1; }
fi
