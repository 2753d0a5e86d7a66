#!/bin/bash
# Copy a round's profile evidence from gpurun_out/prof_$ROUND (tools/profile_round.sh)
# into the tracked profiles/ tree (raw csv of the kernel-stats and the PMC passes
# included, so every number in kernels.json can be recomputed).
set -eu
cd "$(dirname "$0")/.."
R=${ROUND:-r02}
S=gpurun_out/prof_$R
D=profiles/$R
mkdir -p $D/pmc
cp $S/kernels.json $S/bench_kernel_stats.csv $D/
for f in $S/bench_under_rocprof.json $S/bench.json; do [ -f "$f" ] && cp "$f" $D/; done
for sub in traffic sq calib; do
  find $S/$sub -name '*counter_collection.csv' | while read -r f; do
    cp "$f" "$D/pmc/${sub}_$(basename "$f")"
  done
done
echo "$D updated"
