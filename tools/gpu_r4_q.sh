# Round 4 call Q: price the pose kernel's share of the headline mix
# (tools/mix_probe.py: pose on / off, trial groups 1 / 2, 2 / 4 pipelines)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for A in "--pose on" "--pose off" "--pose on --groups 2" "--pose on --pipes 4" "--pose on --pose-chunk 64" "--pose on --pose-chunk 128"; do
    timeout -k 10 200 python tools/mix_probe.py $A 2>/dev/null || exit 1
  done
done
