# inertial kernel iteration: parity tests, phase stamps, per-frame latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_inertial.py tests/test_gpu_track_inertial.py tests/test_gpu_stereo.py tests/test_gpu_match.py tests/test_gpu_bow.py > gpurun_out/inert_tests.log 2>&1; rc=$?; tail -3 gpurun_out/inert_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 env ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/inertial_stamps.py --mode 0 2>gpurun_out/instamps.err || { tail -3 gpurun_out/instamps.err; exit 1; }
timeout -k 10 300 python tools/bench_latency_inertial.py --frames 16 2>gpurun_out/latinert.err | tail -c 1200 || exit 1
