# Round 4 call D: extractor / pose / inertial parity after the FAST chunked
# survivor list and the near-zero pivot routing; FAST A/B vs round 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_pose.py tests/test_gpu_track.py tests/test_gpu_inertial.py tests/test_gpu_track_inertial.py tests/test_gpu_stereo.py > gpurun_out/r4d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4d_tests.log; [ $rc -eq 0 ] || exit $rc
ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_varB.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extractor.py > gpurun_out/r4d_varB.log 2>&1; rc=$?; echo "varB extractor:"; tail -2 gpurun_out/r4d_varB.log; [ $rc -lt 124 ] || exit $rc
bash tools/valu_ab.sh > gpurun_out/valu_ab.log 2>&1 || { tail -5 gpurun_out/valu_ab.log; exit 1; }
grep -E "liborbgpu|k_fast|k_resize" gpurun_out/valu_ab.log
bash tools/ab_fast.sh > gpurun_out/ab_fast.log 2>&1 || { tail -5 gpurun_out/ab_fast.log; exit 1; }
cut -c1-300 gpurun_out/ab_fast.log
for R in levels fused; do echo "== resize $R, 256 images"; ORBGPU_RESIZE=$R timeout -k 10 120 python tools/prof_stages.py --frames 128 --iters 20 --mode ext 2>/dev/null | tail -c 300 || exit 1; done
echo "== pose single"; timeout -k 10 120 python tools/pose_single.py 2>/dev/null || exit 1
bash tools/gpu_r4_e.sh
