# Round 4: LBA / LIA parity (new solver paths, VertexPose-only key frames,
# windows past the old bounds) + solver A/B timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lia.py > gpurun_out/lba_r4_tests.log 2>&1; rc=$?; tail -40 gpurun_out/lba_r4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lba_solver_ab.py 3 > gpurun_out/lba_solver_ab.log 2>&1; rc=$?; cat gpurun_out/lba_solver_ab.log; exit $rc
