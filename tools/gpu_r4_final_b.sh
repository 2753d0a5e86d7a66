# Round 4 final call B: extractor evidence (PMC passes, bench under rocprof,
# kernels.json) and the bench line, under gpurun_out/prof_r04
set -o pipefail
ROUND=r04 FRAMES=128 bash tools/profile_round.sh
