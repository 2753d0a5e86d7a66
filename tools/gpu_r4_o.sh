# Round 4 call O: LBA / LIA tests (zero-iteration / repeat-call cases, the
# fused host layout, the per-pair inline Schur fold) and timing, fold A/B;
# headline with 2 / 3 / 4 extractor pipelines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
HL="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded"
bash tools/gpu_r4_h.sh || exit 1
for F in launch inline launch inline; do
  for W in lba lia; do X=""; [ $W = lia ] && X="--lia"
    ORBGPU_SCHUR_FOLD=$F timeout -k 10 200 python tools/bench_lba.py $X --calls 30 --cpu-calls 0 > gpurun_out/o_fold_$W.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/o_fold_$W.json'));print('fold $F $W', d['gpu_ms_per_call'])"
  done
done
for P in 2 3 4 2 3 4; do
  timeout -k 10 300 python bench.py $HL --pipes $P > gpurun_out/o_bench_p$P.json 2> gpurun_out/o_bench_p$P.err || { tail -3 gpurun_out/o_bench_p$P.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/o_bench_p$P.json').read().strip().splitlines()[-1]);print('pipes $P', d['value'], d['ms_per_step'])"
done
