#!/bin/bash
# Interleaved A/B of library builds (ORBGPU_LIB) on one box: the isolated
# extractor stage times (tools/prof_stages.py) and the headline bench line
# (side lines off), ROUNDS times each, in alternation.
#   LIBS="orb_slam_fusion_amd/lib/liborbgpu_d1.so orb_slam_fusion_amd/lib/liborbgpu.so" ROUNDS=2 bash tools/ab_bench.sh
# BENCH_ARGS: extra bench.py arguments; ARGSETS="a;b;c": one bench per set
# (per library), e.g. ARGSETS="--phase-stage -1;--phase-stage 2"
# Every run's stderr is kept in gpurun_out/ab_<n>.err (named in the output).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
n_run=0
errlog() { n_run=$((n_run + 1)); echo "gpurun_out/ab_${n_run}.err"; }
NOSIDE="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded"
for i in $(seq 1 "${ROUNDS:-2}"); do
  for L in ${LIBS:-orb_slam_fusion_amd/lib/liborbgpu.so}; do
    [ -f "$L" ] || { echo "missing $L"; exit 1; }
    echo "== $L round $i"
    if [ "${STAGES:-1}" = "1" ]; then
      E=$(errlog)
      timeout -k 10 120 env ORBGPU_LIB="$L" python tools/prof_stages.py --frames 128 --iters 20 --mode ext 2>"$E" | tail -c 500 \
        || { echo "prof_stages failed (stderr: $E)"; tail -n 20 "$E"; exit 1; }
      echo
    fi
    IFS=';' read -r -a SETS <<< "${ARGSETS:- }"
    for A in "${SETS[@]}"; do
      # shellcheck disable=SC2086
      E=$(errlog)
      timeout -k 10 200 env ORBGPU_LIB="$L" python bench.py --steps 20 $NOSIDE ${BENCH_ARGS:-} $A 2>"$E" \
        | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench [$A]', d['value'], d['ms_per_step'])" \
        || { echo "bench failed (stderr: $E)"; tail -n 20 "$E"; exit 1; }
    done
  done
done
