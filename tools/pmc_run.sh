#!/bin/bash
# PMC passes over the isolated extractor chain (one counter group per pass;
# counters are collected with --kernel-trace only, never with sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="${PROF_ARGS:---iters 3 --mode ext}"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $counters --kernel-trace -d $OUT -o pass$i --output-format csv \
    -- python3 tools/prof_stages.py $ARGS > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done < "${PMC_GROUPS:-tools/pmc_groups.txt}"
echo "passes: $i"
