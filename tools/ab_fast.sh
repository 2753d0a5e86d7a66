# A/B/C timing of the extractor stages across library builds (ORBGPU_LIB)
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/ab_fast.err
set -o pipefail
for i in 1 2 3; do
  for L in orb_slam_fusion_amd/lib/liborbgpu_base.so orb_slam_fusion_amd/lib/liborbgpu_varB.so orb_slam_fusion_amd/lib/liborbgpu.so; do
    [ -f $L ] || continue
    echo "== $L"; timeout -k 10 120 env ORBGPU_LIB=$L python tools/prof_stages.py --frames 128 --iters 20 --mode ext 2>>gpurun_out/ab_fast.err | tail -c 400 || exit 1
  done
done
