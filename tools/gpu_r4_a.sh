# Round 4 call A: extractor / pose / LBA / LIA parity, FAST + pose A/B against
# the round-3 build (liborbgpu_base.so), LBA timing, back-end profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_pose.py tests/test_gpu_track.py > gpurun_out/r4a_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4a_tests.log; [ $rc -eq 0 ] || exit $rc
for L in liborbgpu_base liborbgpu; do
  echo "== $L pose single"; ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 120 python tools/pose_single.py 2>/dev/null || exit 1
  echo "== $L pose batch"; ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 120 python tools/prof_stages.py --mode pose 2>/dev/null | tail -c 300 || exit 1
done
bash tools/valu_ab.sh > gpurun_out/valu_ab.log 2>&1 || { tail -5 gpurun_out/valu_ab.log; exit 1; }
grep -E "liborbgpu|k_fast|k_describe|k_pose" gpurun_out/valu_ab.log
bash tools/ab_fast.sh > gpurun_out/ab_fast.log 2>&1 || { tail -5 gpurun_out/ab_fast.log; exit 1; }
cut -c1-400 gpurun_out/ab_fast.log
PROF=1 bash tools/gpu_lba_r4.sh
