#!/bin/bash
# HBM traffic per extractor-stage launch for bench.py's roofline.traffic:
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md: the
# TCC counters cannot share a pass; FETCH_SIZE is doubled on gfx950), over the
# workload of one bench pipeline launch (32 stereo frames = 64 images).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic
rm -rf $OUT; mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d $OUT -o $c --output-format csv \
    -- python3 tools/prof_stages.py --frames 32 --iters 3 --mode ext > $OUT/$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
python3 tools/pmc_traffic.py $OUT profiles/pmc_traffic.json
