# Round 4 call P: LBA / LIA after reverting the inline fold and the fused
# edge-image walk (tests + timing + layout trace), sums without the later
# builds' maxima
set -o pipefail
bash tools/gpu_r4_h.sh || exit 1
for W in lba lia lba lia; do X=""; [ $W = lia ] && X="--lia"
  timeout -k 10 200 python tools/bench_lba.py $X --calls 30 --cpu-calls 0 > gpurun_out/p_$W.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/p_$W.json'));print('$W', d['gpu_ms_per_call'])"
done
