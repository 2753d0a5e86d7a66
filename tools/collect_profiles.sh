#!/bin/bash
# Copy a round's profile evidence from gpurun_out/prof_$ROUND (tools/profile_round.sh)
# into the tracked profiles/ tree.
set -eu
cd "$(dirname "$0")/.."
R=${ROUND:-r01}
S=gpurun_out/prof_$R
mkdir -p profiles/$R/pmc_traffic
cp $S/bench_kernel_stats.csv $S/bench_kernel_stats.txt $S/bench_under_rocprof.json $S/bench.json \
   $S/pmc_sq.txt $S/pmc_sq.json profiles/$R/
cp $S/pmc_traffic/*.csv profiles/$R/pmc_traffic/
cp $S/pmc_traffic.json profiles/pmc_traffic.json
cp $S/pmc_sq.json profiles/pmc_sq.json
echo "profiles/$R updated"
