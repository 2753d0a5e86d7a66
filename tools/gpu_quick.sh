#!/bin/bash
# Parity tests + isolated stage timings (one gpurun call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/prof_stages.py ${PROF_ARGS:-} > gpurun_out/stages.json 2> gpurun_out/stages.err
rc=$?
echo "stages rc=$rc"; cat gpurun_out/stages.json; tail -3 gpurun_out/stages.err
exit $rc
