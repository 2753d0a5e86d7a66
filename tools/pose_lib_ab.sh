# Pose parity tests, then batch and single-problem timing for two library
# builds (ORBGPU_LIB): liborbgpu_base.so vs the current liborbgpu.so
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/pose_lib_ab.err
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pose.py tests/test_gpu_track.py > gpurun_out/pose_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pose_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in liborbgpu_base liborbgpu; do
    echo "== $L"
    ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 120 python tools/prof_stages.py --mode pose 2>>gpurun_out/pose_lib_ab.err | tail -c 300 || exit 1
    ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 120 python tools/pose_single.py --frames 40 2>>gpurun_out/pose_lib_ab.err || exit 1
  done
done
