#!/bin/bash
# One gpurun call: GPU parity tests, then (only if nothing crashed) a short
# bench.  Every GPU step has its own time limit; a crash/timeout stops the
# script.  Logs go to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
ok_rc $rc || exit $rc

if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --cpu-seconds 6} \
    > gpurun_out/bench.log 2>&1
  rc=$?
  echo "bench rc=$rc"; tail -n 5 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
