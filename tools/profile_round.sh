#!/bin/bash
# Evidence for a round (one gpurun call): PMC traffic of the roofline kernel,
# rocprofv3 kernel-trace stats of the bench command itself, and the bench line.
#   ROUND=r01 bash tools/profile_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r01}
mkdir -p gpurun_out profiles/$R
bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { echo "pmc traffic failed"; tail -5 gpurun_out/pmc_traffic.log; exit 1; }
cp profiles/pmc_traffic.json gpurun_out/ 2>/dev/null
rm -rf gpurun_out/bench_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/bench_prof -o bench \
  -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo "rocprof bench failed"; tail -5 gpurun_out/bench_prof.log; exit 1; }
f=$(find gpurun_out/bench_prof -name '*kernel_stats.csv' | head -n1)
cp "$f" gpurun_out/bench_kernel_stats.csv  # copy into profiles/$R/ locally (only gpurun_out/ returns)
python3 tools/kstats.py "$f" > profiles/$R/bench_kernel_stats.txt
grep '^{' gpurun_out/bench_prof.log | tail -1 > profiles/$R/bench_under_rocprof.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_full.log; exit 1; }
grep '^{' gpurun_out/bench_full.log | tail -1 > profiles/$R/bench.json
cat profiles/$R/bench_kernel_stats.txt
cat profiles/$R/bench.json
