#!/bin/bash
# Copy a round's profile evidence from gpurun_out/prof_$ROUND (tools/profile_round.sh)
# into the tracked profiles/ tree: the JSON summaries and the kernel-stats CSV as
# files, the raw PMC counter CSVs compressed (pmc_raw.tar.gz), so every number in
# kernels.json can be recomputed without bloating the history.
set -eu
cd "$(dirname "$0")/.."
R=${ROUND:-r02}
S=gpurun_out/prof_$R
D=profiles/$R
mkdir -p $D
cp $S/kernels.json $S/bench_kernel_stats.csv $D/
for f in $S/bench_under_rocprof.json $S/bench.json $S/vmem.json; do [ -f "$f" ] && cp "$f" $D/; done
T=$(mktemp -d)
for sub in traffic sq calib; do
  find $S/$sub -name '*counter_collection.csv' | while read -r f; do
    cp "$f" "$T/${sub}_$(basename "$f")"
  done
done
tar czf $D/pmc_raw.tar.gz -C $T .
rm -rf "$T"
echo "$D updated"
