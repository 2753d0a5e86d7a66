#!/bin/bash
# Per-kernel durations of the isolated extractor/pose chain.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt -o kt -- python3 tools/prof_stages.py --iters 20 "$@" > gpurun_out/kt.log 2>&1
f=$(find gpurun_out/kt -name '*kernel_stats.csv' | head -n1)
cut -d, -f1-8 "$f"
