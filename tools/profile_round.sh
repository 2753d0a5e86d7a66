#!/bin/bash
# Evidence for a round (one gpurun call), staged under gpurun_out/prof_$ROUND/
# (only gpurun_out/ comes back from the box; tools/collect_profiles.sh copies
# it into profiles/$ROUND/ here):
#   * pmc_traffic.json + csv: FETCH_SIZE / WRITE_SIZE per extractor stage launch
#     (separate passes), read by bench.py's roofline.traffic;
#   * pmc_sq.txt / .json: SQ instruction-mix and VALU-busy counters per kernel;
#   * bench_kernel_stats.{csv,txt} + bench_under_rocprof.json: rocprofv3
#     --kernel-trace --stats of the bench command itself;
#   * bench.json: the bench line without the profiler.
#   ROUND=r01 bash tools/profile_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r01}
O=gpurun_out/prof_$R
rm -rf "$O"; mkdir -p "$O"
bash tools/pmc_traffic.sh > "$O/pmc_traffic.log" 2>&1 || { echo "pmc traffic failed"; tail -5 "$O/pmc_traffic.log"; exit 1; }
cp profiles/pmc_traffic.json "$O/"
mkdir -p "$O/pmc_traffic" && cp gpurun_out/pmc_traffic/*counter_collection.csv "$O/pmc_traffic/" 2>/dev/null
rm -rf gpurun_out/pmc
PMC_GROUPS=tools/pmc_groups_sq2.txt bash tools/pmc_run.sh > "$O/pmc_sq.log" 2>&1 || { echo "pmc sq failed"; tail -5 "$O/pmc_sq.log"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc --json "$O/pmc_sq.json" > "$O/pmc_sq.txt"
rm -rf gpurun_out/bench_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/bench_prof -o bench \
  -- python3 bench.py --no-cpu-baseline --no-lba --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency > "$O/bench_prof.log" 2>&1 || { echo "rocprof bench failed"; tail -5 "$O/bench_prof.log"; exit 1; }
f=$(find gpurun_out/bench_prof -name '*kernel_stats.csv' | head -n1)
cp "$f" "$O/bench_kernel_stats.csv"
python3 tools/kstats.py "$f" > "$O/bench_kernel_stats.txt"
grep '^{' "$O/bench_prof.log" | tail -1 > "$O/bench_under_rocprof.json"
timeout -k 10 400 python3 bench.py > "$O/bench_full.log" 2>&1 || { echo "bench failed"; tail -5 "$O/bench_full.log"; exit 1; }
grep '^{' "$O/bench_full.log" | tail -1 > "$O/bench.json"
cat "$O/bench_kernel_stats.txt"
cat "$O/bench.json"
