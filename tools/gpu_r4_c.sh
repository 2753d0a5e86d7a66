# Round 4 call C: LBA / LIA parity + timing + kernel-trace stats (Schur rework)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lia.py > gpurun_out/lba_r4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lba_r4_tests.log; [ $rc -eq 0 ] || exit $rc
for W in lba lia; do
  X=""; [ $W = lia ] && X="--lia"
  timeout -k 10 200 python tools/bench_lba.py $X --calls 20 --cpu-calls 0 > gpurun_out/bench_$W.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_$W.json'));print('$W', {k:d[k] for k in d if 'ms' in k})"
  rm -rf gpurun_out/kt_$W
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_$W -o kt -- python3 tools/bench_lba.py $X --calls 10 --cpu-calls 0 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/kt_$W -name "*kernel_stats.csv" | head -1); python -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('  %-40s n=%5s avg_us=%8.2f' % (r['Name'].split('(')[0].split('::')[-1][:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
