#!/bin/bash
# Interleaved A/B of the LBA step variants (C4 and LIA ms per call):
# base = another library build (build/wt0, when present), launch-fold = this
# tree's with ORBGPU_SCHUR_FOLD=launch, inline-fold = this tree's default.
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  c4=$(env "$@" timeout -k 10 200 python tools/bench_lba.py --calls 20 --cpu-calls 0 2>>gpurun_out/fold_ab.err \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['gpu_ms_per_call'])") || return 1
  lia=$(env "$@" timeout -k 10 200 python tools/bench_lba.py --lia --calls 20 --cpu-calls 0 2>>gpurun_out/fold_ab.err \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['gpu_ms_per_call'])") || return 1
  echo "$name c4=$c4 lia=$lia"
}
for i in $(seq 1 "${ROUNDS:-3}"); do
  [ -f build/wt0/liborbgpu.so ] && { run base ORBGPU_LIB=build/wt0/liborbgpu.so || exit 1; }
  run launch-fold ORBGPU_SCHUR_FOLD=launch || exit 1
  run inline-fold ORBGPU_X=0 || exit 1
done
