# Interleaved A/B of library builds on the inertial batch / single-problem
# timing (tools/bench_inertial.py, modes 0 and 1), with a bit-identity hash of
# the batch results:  LIBS="liborbgpu_base liborbgpu" ROUNDS=3 bash tools/inert_ab.sh
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/inert_ab.err
for i in $(seq ${ROUNDS:-3}); do
  for L in ${LIBS:-liborbgpu_base liborbgpu}; do
    for M in ${MODES:-0 1}; do
      echo "== $L mode $M"
      ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 80 python tools/bench_inertial.py --mode $M 2>>gpurun_out/inert_ab.err | tail -c 420 || exit 1
    done
  done
done
