# Round 4 final call B: LBA / LIA parity after the link-record change, then
# the extractor evidence (PMC passes, bench under rocprof, kernels.json) and
# the bench line, under gpurun_out/prof_r04
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lia.py > gpurun_out/fb_tests.log 2>&1; rc=$?; tail -1 gpurun_out/fb_tests.log; [ $rc -eq 0 ] || exit $rc
ROUND=r04 FRAMES=128 bash tools/profile_round.sh
