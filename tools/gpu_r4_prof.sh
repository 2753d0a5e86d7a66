# Round 4 evidence: extractor PMC passes + bench under rocprof + kernels.json
# + the bench line (tools/profile_round.sh), then the back-end passes
# (tools/ba_prof.sh)
set -o pipefail
ROUND=r04 RUN_BENCH=1 bash tools/profile_round.sh || exit 1
ROUND=r04 bash tools/ba_prof.sh || exit 1
