# Extractor + LBA/LIA parity tests, then stage timings (extractor) and
# per-call LBA / LIA timings for liborbgpu_base.so vs the current liborbgpu.so
mkdir -p gpurun_out  # stderr of every run is kept in gpurun_out/ext_lba_ab.err
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lia.py > gpurun_out/ext_lba_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ext_lba_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in liborbgpu_base liborbgpu; do
    echo "== $L"

    ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 200 python tools/bench_lba.py --calls 20 --cpu-calls 0 2>>gpurun_out/ext_lba_ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k: v for k, v in d.items() if not isinstance(v, dict)})" || exit 1
    ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so timeout -k 10 200 python tools/bench_lba.py --lia --calls 20 --cpu-calls 0 2>>gpurun_out/ext_lba_ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k: v for k, v in d.items() if not isinstance(v, dict)})" || exit 1
  done
done
