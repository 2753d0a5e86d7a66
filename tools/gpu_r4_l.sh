# Round 4 call L: k_blur rows of loads in flight (ORB_BLUR_PF 8 / 4 / 6:
# 73 / 62 / 68 VGPRs) -- blur bit-exact per variant, stage times and the
# headline mix A/B interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
HL="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded"
for L in liborbgpu_pf4 liborbgpu_pf6; do
  ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py > gpurun_out/l_ext_$L.log 2>&1; rc=$?; echo "$L: $(tail -1 gpurun_out/l_ext_$L.log)"; [ $rc -eq 0 ] || exit $rc
done
for L in liborbgpu liborbgpu_pf4 liborbgpu_pf6; do
  echo "== $L"; ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 120 python tools/prof_stages.py --frames 128 --iters 20 --mode ext 2>/dev/null | tail -c 300 || exit 1
done
for L in liborbgpu liborbgpu_pf4 liborbgpu_pf6 liborbgpu liborbgpu_pf4 liborbgpu_pf6; do
  ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 300 python bench.py $HL > gpurun_out/l_bench_$L.json 2> gpurun_out/l_bench_$L.err || { tail -3 gpurun_out/l_bench_$L.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/l_bench_$L.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'])"
done
