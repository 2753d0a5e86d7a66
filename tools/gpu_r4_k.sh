# Round 4 call K: call J (k_describe A/B) + call H (LBA / LIA parity and
# timing: the first build's link forms now from k_lba_begin)
set -o pipefail
bash tools/gpu_r4_h.sh || exit 1
bash tools/gpu_r4_j.sh || exit 1
