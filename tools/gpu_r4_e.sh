# Round 4 call E: LBA / LIA parity with the point-range Schur (default), the
# three Schur paths A/B (ORBGPU_SCHUR), kernel-trace stats of the default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for W in lba lia; do
  X=""; [ $W = lia ] && X="--lia"
  for M in pair band split; do
    ORBGPU_SCHUR=$M timeout -k 10 200 python tools/bench_lba.py $X --calls 20 --cpu-calls 0 > gpurun_out/bench_${W}_$M.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/bench_${W}_$M.json'));print('$W $M', {k:d[k] for k in d if 'ms' in k or 'chi2' in k or 'err_end' in k})"
  done
  rm -rf gpurun_out/kt_$W
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_$W -o kt -- python3 tools/bench_lba.py $X --calls 10 --cpu-calls 0 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/kt_$W -name "*kernel_stats.csv" | head -1); python -c "
import csv,re
for r in csv.DictReader(open('$f')):
    n=re.sub(r'\(orbgpu::LbaArgs.*','',r['Name']).replace('void ','').replace('orbgpu::(anonymous namespace)::','')
    print('  %-40s n=%5s avg_us=%8.2f' % (n[:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
for NF in 18 25; do timeout -k 10 60 ./build/lba_solve_bench $NF 200 || exit 1; done
ORBGPU_LBA_TRACE=1 timeout -k 10 100 python tools/bench_lba.py --calls 5 --cpu-calls 0 2> gpurun_out/trace_lba.log > /dev/null || exit 1; tail -2 gpurun_out/trace_lba.log
ORBGPU_LBA_TRACE=1 timeout -k 10 100 python tools/bench_lba.py --lia --calls 5 --cpu-calls 0 2> gpurun_out/trace_lia.log > /dev/null || exit 1; tail -2 gpurun_out/trace_lia.log
