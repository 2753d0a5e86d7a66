# Round 4 call J: k_describe with its constant-table loads in flight with the
# patch loads and the level found in one scalar round trip -- extractor
# bit-exact, stage times and headline A/B against the previous build (_base)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
HL="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-latency-inertial --no-c5 --no-lba-sharded"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_track.py > gpurun_out/j_ext.log 2>&1; rc=$?; tail -1 gpurun_out/j_ext.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in liborbgpu_base liborbgpu; do
    echo "== $L"; ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 120 python tools/prof_stages.py --frames 128 --iters 20 --mode ext 2>/dev/null | tail -c 400 || exit 1
  done
done
for L in liborbgpu_base liborbgpu liborbgpu_base liborbgpu; do
  ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 300 python bench.py $HL > gpurun_out/j_bench_$L.json 2> gpurun_out/j_bench_$L.err || { tail -3 gpurun_out/j_bench_$L.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/j_bench_$L.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'], d.get('timed_region_s'))"
done
