# Headline sweep over launch-group size and extractor pipelines (bench.py, side lines off)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/sweep
NS="--no-cpu-baseline --no-lba --no-lia --no-stereo --no-match --no-bow --no-inertial --no-track --no-latency --no-c5 --no-lba-sharded --steps 10 --warmup 3"
# CFGS="64,2 256,2" : stereo frames per launch group, pipelines
for cfg in ${CFGS:-64,2 256,2}; do
  cfg=${cfg/,/ }
  set -- $cfg
  timeout -k 10 200 python3 bench.py $NS --batch $1 --pipes $2 > gpurun_out/sweep/b_$1_$2.json 2> gpurun_out/sweep/b_$1_$2.err || exit 1
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sweep/b_$1_$2.json').read().splitlines()[0]);print('$1 $2',d['value'],d['ms_per_step'])"
done
