set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 env ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/pose_stamps.py > gpurun_out/pose_stamps.json 2>gpurun_out/pose_stamps.err || { tail -3 gpurun_out/pose_stamps.err; exit 1; }
cat gpurun_out/pose_stamps.json
timeout -k 10 120 env ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/stamps.py > gpurun_out/fast_stamps.json 2>gpurun_out/fast_stamps.err || { tail -3 gpurun_out/fast_stamps.err; exit 1; }
cat gpurun_out/fast_stamps.json
ROUND=r03 timeout -k 10 900 bash tools/ba_prof.sh > gpurun_out/ba_prof.log 2>&1 || { tail -5 gpurun_out/ba_prof.log; exit 1; }
tail -3 gpurun_out/ba_prof.log
