# Round 4 call S: the back substitution with split FMA chains -- solve phase
# clocks and residual, LBA / LIA tests and timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for NF in 18 25; do timeout -k 10 60 ./build/lba_solve_bench $NF 200 > gpurun_out/s_solve_nf$NF.json || exit 1; cat gpurun_out/s_solve_nf$NF.json; echo; done
bash tools/gpu_r4_h.sh || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lba.py -k "solver or bound or large or grid" > gpurun_out/s_solvers.log 2>&1; rc=$?; tail -1 gpurun_out/s_solvers.log; [ $rc -eq 0 ] || exit $rc
