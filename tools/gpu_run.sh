#!/bin/bash
# The one gpurun entry point: every step optional, each under its own time
# limit, chained so the first failure ends the call (no GPU step after a
# fault, abort or timeout).  Logs under gpurun_out/$TAG*.
#
#   TESTS="tests -m gpu"      pytest targets/args ("" = skip; default: the GPU suite)
#   SMOKE=1                   __graft_entry__.smoke()
#   BENCH="--steps 20 ..."    bench.py with these args (unset = skip)
#   PROFILE=r05               tools/profile_round.sh (extractor PMC + rocprof stats + bench)
#   BAPROF=r05                tools/ba_prof.sh (LBA / LIA PMC + stats)
#   STEPS="cmd1;;cmd2"        extra commands, ';;'-separated, each under timeout 300
#   TAG=x                     log-name prefix (default run)
#
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'TAG=a TESTS="tests/test_gpu_lba.py" bash tools/gpu_run.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=gpurun_out/${TAG:-run}
step() {  # name, limit (s), command...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "${T}_$name.log" 2>&1
  local rc=$?
  tail -c 1500 "${T}_$name.log" | tail -n 6
  [ $rc -eq 0 ] || { echo "!! $name failed rc=$rc"; exit $rc; }
}
if [ "${TESTS-tests -m gpu}" != "" ]; then
  # shellcheck disable=SC2086
  step tests "${TEST_LIMIT:-1000}" python -u -m pytest -x -q --timeout 240 --timeout-method thread ${TESTS-tests -m gpu}
fi
[ -n "${SMOKE:-}" ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [ -n "${BENCH+x}" ]; then
  # shellcheck disable=SC2086
  step bench 600 python bench.py $BENCH
fi
if [ -n "${STEPS:-}" ]; then
  i=0
  while IFS= read -r cmd; do
    [ -z "$cmd" ] && continue
    i=$((i + 1))
    step "step$i" 300 bash -c "$cmd"
  done < <(printf '%s\n' "${STEPS//;;/$'\n'}")
fi
[ -n "${PROFILE:-}" ] && step profile 1100 env ROUND="$PROFILE" bash tools/profile_round.sh
[ -n "${BAPROF:-}" ] && step baprof 900 env ROUND="$BAPROF" bash tools/ba_prof.sh
exit 0
