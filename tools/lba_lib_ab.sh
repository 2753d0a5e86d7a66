# Interleaved A/B of library builds on the C4 LocalBundleAdjustment and the
# LocalInertialBA calls (tools/bench_lba.py):
#   LIBS="liborbgpu_base liborbgpu" ROUNDS=2 bash tools/lba_lib_ab.sh
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/lba_lib_ab.err
for i in $(seq ${ROUNDS:-2}); do
  for L in ${LIBS:-liborbgpu_base liborbgpu}; do
    for M in "" "--lia"; do
      ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 200 python tools/bench_lba.py $M --calls 30 --cpu-calls 0 2>>gpurun_out/lba_lib_ab.err \
        | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L $M', d.get('gpu_ms_per_call'), d.get('lm_iterations'), d.get('chi2_gpu'))" || exit 1
    done
  done
done
