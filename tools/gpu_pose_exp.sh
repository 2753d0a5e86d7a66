# PoseOptimization experiment: parity, phase stamps, batch and single-frame timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pose.py tests/test_gpu_track.py > gpurun_out/pose_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pose_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 env ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/pose_stamps.py 2>gpurun_out/pose_stamps.err || { tail -3 gpurun_out/pose_stamps.err; exit 1; }
timeout -k 10 120 python tools/prof_stages.py --mode pose 2>/dev/null | tail -c 600 || exit 1
timeout -k 10 200 python tools/bench_latency.py --frames 40 2>/dev/null | tail -c 500 || exit 1
timeout -k 10 120 python tools/pose_single.py 2>gpurun_out/pose_single.err || { tail -3 gpurun_out/pose_single.err; exit 1; }
