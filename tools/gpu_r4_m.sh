# Round 4 call M: k_resize staging without index divisions (ORB_RESIZE_STAGE_FAST;
# _rs0 = the general path) and k_blur 6 rows in flight -- extractor bit-exact,
# VALU counts, stage times, headline A/B interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
HL="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_track.py > gpurun_out/m_ext.log 2>&1; rc=$?; tail -1 gpurun_out/m_ext.log; [ $rc -eq 0 ] || exit $rc
LIBS="liborbgpu_rs0 liborbgpu" bash tools/valu_ab.sh > gpurun_out/m_valu.log 2>&1 || { tail -5 gpurun_out/m_valu.log; exit 1; }
grep -E "liborbgpu|k_resize|k_blur" gpurun_out/m_valu.log
for L in liborbgpu_rs0 liborbgpu; do
  echo "== $L"; ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 120 python tools/prof_stages.py --frames 128 --iters 20 --mode ext 2>/dev/null | tail -c 300 || exit 1
done
for L in liborbgpu_rs0 liborbgpu liborbgpu_rs0 liborbgpu; do
  ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 300 python bench.py $HL > gpurun_out/m_bench_$L.json 2> gpurun_out/m_bench_$L.err || { tail -3 gpurun_out/m_bench_$L.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/m_bench_$L.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'])"
done
