#!/bin/bash
# Interleaved per-frame latency A/B on one box (tools/latency.cc): the
# single-image dataflow launch (default) against the per-stage graph path
# (ORBGPU_SINGLE=graph), stereo pairs on two threads and one image on one
# thread, ROUNDS times each.  Optional LIBS="dir1 dir2": extra library
# builds (a liborbgpu.so in each dir, via LD_LIBRARY_PATH).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 "${ROUNDS:-3}"); do
  for mode in stereo mono; do
    m=""; [ "$mode" = mono ] && m=mono
    for v in df graph ${LIBS:-}; do
      case $v in
        df) env=() ;;
        graph) env=(ORBGPU_SINGLE=graph) ;;
        *) env=(LD_LIBRARY_PATH="$v") ;;
      esac
      out=$(timeout -k 5 60 env "${env[@]}" build/latency 200 10 $m 2>>gpurun_out/lat_ab.err) || { echo "latency failed ($v $mode)"; exit 1; }
      echo "$i $mode $v $(echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if k.startswith('gpu_')})")"
    done
  done
done
