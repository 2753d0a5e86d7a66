#!/bin/bash
# Interleaved per-frame latency A/B on one box (tools/latency.cc): stereo
# pairs on two threads and one image on one thread, ROUNDS times each, for
# every variant of VARIANTS ("name:ENV=v ENV2=w ..."; default: the dataflow
# launch against the per-stage graph path, ORBGPU_SINGLE=graph).  A variant's
# env may name another library build through LD_LIBRARY_PATH.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"df: graph:ORBGPU_SINGLE=graph"}
for i in $(seq 1 "${ROUNDS:-3}"); do
  for mode in ${MODES:-stereo mono}; do
    m=""; [ "$mode" != stereo ] && m=$mode
    for v in $VARIANTS; do
      name=${v%%:*}; envs=${v#*:}
      # shellcheck disable=SC2086
      out=$(timeout -k 5 60 env ${envs//,/ } build/latency 200 10 $m 2>>gpurun_out/lat_ab.err) \
        || { echo "latency failed ($name $mode)"; tail -n 5 gpurun_out/lat_ab.err; exit 1; }
      echo "$i $mode $name $(echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if k.startswith('gpu_')})")"
    done
  done
done
