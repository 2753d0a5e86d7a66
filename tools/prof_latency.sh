#!/bin/bash
# rocprofv3 kernel traces of the two per-frame latency legs (C++ callers of the
# C ABI): build/latency pair (stereo extraction + PoseOptimization) and
# build/latency_inertial (its inputs dumped by tools/bench_latency_inertial.py);
# the --stats summaries land in gpurun_out/prof_lat_$ROUND/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof_lat_${ROUND:-r06}
rm -rf "$O"; mkdir -p "$O"
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $O/pair -o pair \
  -- build/latency 200 10 pair > $O/pair.json 2> $O/pair.err || { echo "pair failed"; tail -5 $O/pair.err; exit 1; }
ORBGPU_LATIN_DUMP=$O/latin.bin timeout -k 10 300 python3 tools/bench_latency_inertial.py --frames 16 --cpu-frames 0 \
  > $O/latency_inertial.json 2> $O/li.err || { echo "dump failed"; tail -5 $O/li.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $O/inertial -o inertial \
  -- build/latency_inertial $O/latin.bin 3 stereo 4 > $O/inertial.json 2> $O/inertial.err \
  || { echo "inertial failed"; tail -5 $O/inertial.err; exit 1; }
rm -f $O/latin.bin
for leg in pair inertial; do
  f=$(find $O/$leg -name '*kernel_stats.csv' | head -n1)
  [ -n "$f" ] && cp "$f" $O/${leg}_kernel_stats.csv
  f=$(find $O/$leg -name '*memory_copy_stats.csv' | head -n1)
  [ -n "$f" ] && cp "$f" $O/${leg}_memory_copy_stats.csv
done
ls $O
