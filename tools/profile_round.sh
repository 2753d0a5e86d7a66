#!/bin/bash
# Evidence for a round (one gpurun call), staged under gpurun_out/prof_$ROUND/
# (only gpurun_out/ comes back from the box; tools/collect_profiles.sh copies
# it into profiles/$ROUND/ here):
#   * FETCH_SIZE / WRITE_SIZE passes (separate: the TCC block cannot hold
#     both) over tools/prof_stages.py -> HBM bytes per stage launch;
#   * an SQ pass over the same workload and over build/valu_calib (the
#     VALU-saturating calibration kernel) -> calibrated VALU-busy;
#   * rocprofv3 --kernel-trace --stats of the bench command itself;
#   * kernels.json (tools/pmc_kernels.py): what bench.py's roofline reads;
#   * bench.json: the bench line without the profiler.
#   ROUND=r05 bash tools/profile_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r02}
O=gpurun_out/prof_$R
rm -rf "$O"; mkdir -p "$O"
# the bench's launch size: 1920 stereo frames = 3840 images a launch (four
# pipelines of the 7680-frame group, bench.py's default)
FR=${FRAMES:-1920}
WL="tools/prof_stages.py --frames $FR --iters 5 --mode both"
SQ="SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c --kernel-trace -d $O/traffic -o $c --output-format csv \
    -- python3 $WL > $O/traffic_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/traffic_$c.log; exit 1; }
done
echo "traffic passes ok"
timeout -k 10 180 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq -o sq --output-format csv \
  -- python3 $WL > $O/sq.log 2>&1 || { echo "pmc sq failed"; tail -5 $O/sq.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc $SQ --kernel-trace -d $O/calib -o calib --output-format csv \
  -- ./build/valu_calib 5 > $O/calib.log 2>&1 || { echo "pmc calib failed"; tail -5 $O/calib.log; exit 1; }
echo "sq passes ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/bench_prof -o bench \
  -- python3 bench.py --no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial \
     --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded > $O/bench_under_rocprof.json 2> $O/bench_prof.err \
  || { echo "rocprof bench failed"; tail -5 $O/bench_prof.err; exit 1; }
f=$(find $O/bench_prof -name '*kernel_stats.csv' | head -n1)
cp "$f" $O/bench_kernel_stats.csv
python3 tools/pmc_kernels.py --traffic $O/traffic --sq $O/sq --calib $O/calib \
  --stats $O/bench_kernel_stats.csv --images-per-launch $((2 * FR)) --out $O/kernels.json > $O/kernels.log 2>&1 \
  || { echo "summary failed"; tail -5 $O/kernels.log; exit 1; }
echo "kernels.json ok"
if [ "${VMEM:-1}" = "1" ]; then
  # the vector-memory pipeline groups over the same
  # workload, reduced per kernel and merged into kernels.json under "vmem"
  rm -rf gpurun_out/pmc
  PMC_GROUPS=tools/pmc_groups_vmem.txt PROF_ARGS="--frames $FR --iters 3 --mode ext" bash tools/pmc_run.sh \
    > $O/vmem_passes.log 2>&1 || { echo "vmem passes failed"; tail -5 $O/vmem_passes.log; exit 1; }
  python3 tools/pmc_vmem.py gpurun_out/pmc --out $O/vmem.json > $O/vmem.log 2>&1 \
    || { echo "vmem summary failed"; tail -5 $O/vmem.log; exit 1; }
  python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
k = json.load(open(f"{o}/kernels.json"))
v = json.load(open(f"{o}/vmem.json"))
k["vmem"] = {n: {kk: vv for kk, vv in d.items() if kk != "counters_per_dispatch"} for n, d in v.items()}
k["vmem_source"] = "tools/pmc_groups_vmem.txt passes (tools/pmc_run.sh) reduced by tools/pmc_vmem.py"
json.dump(k, open(f"{o}/kernels.json", "w"), indent=1)
PY
  echo "vmem ok"
fi
if [ "${RUN_BENCH:-1}" = "1" ]; then
  BENCH_KERNELS_JSON=$O/kernels.json timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err \
    || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
  tail -c 600 $O/bench.json
fi
exit 0
