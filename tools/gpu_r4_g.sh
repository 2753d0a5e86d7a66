# Round 4 call G: FAST NMS by group entries (both survivor-list variants)
# bit-exact + VALU / time / headline A/B; LIA trial states per lane
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
HL="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_track.py > gpurun_out/g_ext.log 2>&1; rc=$?; tail -1 gpurun_out/g_ext.log; [ $rc -eq 0 ] || exit $rc
ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_varB.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py > gpurun_out/g_varB.log 2>&1; rc=$?; echo "varB:"; tail -1 gpurun_out/g_varB.log; [ $rc -lt 124 ] || exit $rc
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_lia.py > gpurun_out/g_lia.log 2>&1; rc=$?; tail -2 gpurun_out/g_lia.log; [ $rc -lt 124 ] || exit $rc
timeout -k 10 120 python tools/lia_relin_diag.py || exit 1
bash tools/valu_ab.sh > gpurun_out/valu_ab.log 2>&1 || { tail -5 gpurun_out/valu_ab.log; exit 1; }
grep -E "liborbgpu|k_fast" gpurun_out/valu_ab.log
bash tools/ab_fast.sh > gpurun_out/ab_fast.log 2>&1 || { tail -5 gpurun_out/ab_fast.log; exit 1; }
cut -c1-200 gpurun_out/ab_fast.log
for L in liborbgpu liborbgpu_varB liborbgpu liborbgpu_varB; do
  ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 300 python bench.py $HL > gpurun_out/g_bench_$L.json 2> gpurun_out/g_bench_$L.err || { tail -3 gpurun_out/g_bench_$L.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/g_bench_$L.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'], d.get('timed_region_s'))"
done
for W in lba lia; do X=""; [ $W = lia ] && X="--lia"; timeout -k 10 200 python tools/bench_lba.py $X --calls 20 --cpu-calls 0 > gpurun_out/g_bench_$W.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/g_bench_$W.json'));print('$W', d['gpu_ms_per_call'])"; done
