set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pose.py tests/test_gpu_inertial.py tests/test_gpu_extractor.py tests/test_gpu_stereo.py tests/test_gpu_track_inertial.py > gpurun_out/lat_tests.log 2>&1; rc=$?; tail -2 gpurun_out/lat_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_latency.py --frames 40 2>/dev/null | tail -c 500 || exit 1
timeout -k 10 300 python tools/bench_latency_inertial.py --frames 16 2>gpurun_out/latinert.err | tail -c 900 || exit 1
timeout -k 10 120 python tools/lat_probe.py 2>/dev/null || exit 1
timeout -k 10 120 env ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/inertial_stamps.py --mode 0 2>gpurun_out/instamps.err || { tail -3 gpurun_out/instamps.err; exit 1; }
