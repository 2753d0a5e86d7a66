# Round 4 call B: extractor / pose / LIA parity, FAST A/B vs round 3, LIA timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_pose.py tests/test_gpu_track.py tests/test_gpu_lia.py tests/test_gpu_stereo.py > gpurun_out/r4b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4b_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/valu_ab.sh > gpurun_out/valu_ab.log 2>&1 || { tail -5 gpurun_out/valu_ab.log; exit 1; }
grep -E "liborbgpu|k_fast" gpurun_out/valu_ab.log
bash tools/ab_fast.sh > gpurun_out/ab_fast.log 2>&1 || { tail -5 gpurun_out/ab_fast.log; exit 1; }
cut -c1-300 gpurun_out/ab_fast.log
timeout -k 10 200 python tools/bench_lba.py --lia --calls 20 --cpu-calls 0 > gpurun_out/bench_lia.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_lia.json'));print({k:d[k] for k in d if 'ms' in k})"
