# A/B of the pose kernel's trial groups: parity tests, batch timing, latency
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/pose_ab.err
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pose.py tests/test_gpu_track.py tests/test_gpu_inertial.py > gpurun_out/pose_tests.log 2>&1; tail -3 gpurun_out/pose_tests.log
for G in 1 2; do
  echo "== G=$G"
  ORBGPU_POSE_GROUPS=$G timeout -k 10 120 python tools/prof_stages.py --mode pose 2>>gpurun_out/pose_ab.err || exit 1
  ORBGPU_POSE_GROUPS=$G timeout -k 10 200 python tools/bench_latency.py --frames 40 2>>gpurun_out/pose_ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k:d[k] for k in d if 'gpu' in k})" || exit 1
done
