# Round 4 call I: LBA / LIA parity + timing after the link blocks moved into
# the trial kernel and the one-wave back-substitution; solve phase clocks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for NF in 18 25; do timeout -k 10 60 ./build/lba_solve_bench $NF 200 > gpurun_out/i_solve_nf$NF.json || exit 1; cat gpurun_out/i_solve_nf$NF.json; echo; done
bash tools/gpu_r4_h.sh
