# Round 4 call H: LBA / LIA parity + timing after the pose-sum split and the
# host layout rework; kernel stats, host phase trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lia.py > gpurun_out/h_tests.log 2>&1; rc=$?; tail -2 gpurun_out/h_tests.log; [ $rc -eq 0 ] || exit $rc
for W in lba lia; do
  X=""; [ $W = lia ] && X="--lia"
  timeout -k 10 200 python tools/bench_lba.py $X --calls 30 --cpu-calls 0 > gpurun_out/h_bench_$W.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/h_bench_$W.json'));print('$W', d['gpu_ms_per_call'])"
  ORBGPU_LBA_TRACE=1 timeout -k 10 100 python tools/bench_lba.py $X --calls 5 --cpu-calls 0 2> gpurun_out/h_trace_$W.log > /dev/null || exit 1; tail -1 gpurun_out/h_trace_$W.log
  rm -rf gpurun_out/kt_$W
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_$W -o kt -- python3 tools/bench_lba.py $X --calls 10 --cpu-calls 0 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/kt_$W -name "*kernel_stats.csv" | head -1); python -c "
import csv,re
for r in csv.DictReader(open('$f')):
    n=re.sub(r'\(orbgpu::LbaArgs.*','',r['Name']).replace('void ','').replace('orbgpu::(anonymous namespace)::','')
    print('  %-40s n=%5s avg_us=%8.2f' % (n[:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
timeout -k 10 120 python tools/pose_single.py || exit 1
