#!/bin/bash
# Back-end (LocalBundleAdjustment / LocalInertialBA) evidence, one gpurun call:
#   * the solve's phase clocks (build/lba_solve_bench, LBA_SOLVE_STAMPS) at
#     n = 108 (C4) and n = 150;
#   * rocprofv3 --kernel-trace --stats of tools/bench_lba.py (LBA and LIA);
#   * PMC passes per kernel over the same commands, each pass its own run:
#     SQ (VALU, MFMA f64 instructions / MOPS / busy cycles, waves, cycles),
#     FETCH_SIZE, WRITE_SIZE (separate: the TCC block cannot hold both);
#   * tools/ba_roofline.py folds them into ba_kernels.json (what bench.py's
#     lba / lia roofline blocks read).
#   ROUND=r03 bash tools/ba_prof.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r03}
O=gpurun_out/ba_$R
rm -rf "$O"; mkdir -p "$O"
if [ -x build/lba_solve_bench ]; then
  for nf in 18 25; do
    timeout -k 5 60 ./build/lba_solve_bench $nf 200 > $O/solve_stamps_nf$nf.json || { echo "solve bench $nf failed"; exit 1; }
    cat $O/solve_stamps_nf$nf.json
  done
fi
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for W in lba lia; do
  X=""; [ $W = lia ] && X="--lia"
  CMD="python3 tools/bench_lba.py $X --calls 10 --cpu-calls 0"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$W/stats -o stats -- $CMD \
    > $O/$W.json 2> $O/$W.err || { echo "$W stats failed"; tail -3 $O/$W.err; exit 1; }
  i=0
  for C in "$SQ GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/$W/p$i -o p$i --output-format csv -- $CMD \
      > $O/$W/p$i.log 2>&1 || { echo "$W pass $i failed"; tail -3 $O/$W/p$i.log; exit 1; }
  done
  echo "$W passes ok"
done
python3 tools/ba_roofline.py --dir $O --out $O/ba_kernels.json > $O/ba_roofline.log 2>&1 \
  || { echo "summary failed"; tail -5 $O/ba_roofline.log; exit 1; }
cat $O/ba_roofline.log
exit 0
