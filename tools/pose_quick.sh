# pose parity + isolated batch timing + the headline (one gpurun call)
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/pose_quick.err
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pose.py tests/test_gpu_track.py > gpurun_out/pose_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pose_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/prof_stages.py --mode pose 2>>gpurun_out/pose_quick.err || exit 1
timeout -k 10 200 python tools/bench_mix.py 2>>gpurun_out/pose_quick.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-c5 --no-lba-sharded > gpurun_out/bench_quick.json 2>>gpurun_out/pose_quick.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'], d['ms_per_step'], {k:v['avg_ms_per_launch'] for k,v in d['roofline']['kernels'].items()})"
