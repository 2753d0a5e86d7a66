# Inertial / BA parity tests, then batch + single-problem inertial timing for
# two library builds (ORBGPU_LIB): liborbgpu_base.so vs the current liborbgpu.so
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/inert_lib_ab.err
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_inertial.py tests/test_gpu_track_inertial.py tests/test_gpu_lia.py tests/test_gpu_lba.py > gpurun_out/inert_tests.log 2>&1; rc=$?; tail -2 gpurun_out/inert_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in liborbgpu_base liborbgpu; do
    echo "== $L"
    ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 200 python tools/bench_inertial.py 2>>gpurun_out/inert_lib_ab.err | tail -c 400 || exit 1
  done
done
