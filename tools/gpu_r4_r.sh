# Round 4 call R: k_octree held to 64 VGPRs (amdgpu_waves_per_eu 8) alone
# (_oct8) and with k_blur at 4 rows in flight (_occ8, 62 VGPRs): extractor
# bit-exact per variant, headline mix A/B interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
HL="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded"
for L in liborbgpu_oct8 liborbgpu_occ8; do
  ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py > gpurun_out/r_ext_$L.log 2>&1; rc=$?; echo "$L: $(tail -1 gpurun_out/r_ext_$L.log)"; [ $rc -eq 0 ] || exit $rc
done
for L in liborbgpu liborbgpu_oct8 liborbgpu_occ8 liborbgpu liborbgpu_oct8 liborbgpu_occ8; do
  ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 300 python bench.py $HL > gpurun_out/r_bench_$L.json 2> gpurun_out/r_bench_$L.err || { tail -3 gpurun_out/r_bench_$L.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r_bench_$L.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'])"
done
