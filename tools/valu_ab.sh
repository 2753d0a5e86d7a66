# SQ instruction counts of the extractor kernels for library builds
# (ORBGPU_LIB; LIBS overrides the list): base / varB / current, same frames
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/valu_ab; rm -rf $O; mkdir -p $O
LIBS=${LIBS:-liborbgpu_base liborbgpu_varB liborbgpu}
for L in $LIBS; do
  [ -f orb_slam_fusion_amd/lib/$L.so ] || continue
  timeout -s KILL 120 env ORBGPU_LIB=orb_slam_fusion_amd/lib/$L.so rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-trace -d $O/$L -o p --output-format csv -- python3 tools/prof_stages.py --frames 32 --iters 5 --mode ext > $O/$L.log 2>&1 || { echo "pmc failed"; tail -3 $O/$L.log; exit 1; }
done
python3 - "$O" $LIBS <<'PY'
import csv, glob, sys, collections
for L in sys.argv[2:]:
    fs = glob.glob(f"{sys.argv[1]}/{L}/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    f = fs[0]
    acc = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].split('::')[-1].split('<')[0]
        if k.startswith('k_'):
            acc[(k, r['Counter_Name'])][0] += float(r['Counter_Value']); acc[(k, r['Counter_Name'])][1] += 1
    print(L)
    for (k, c), (v, n) in sorted(acc.items()):
        print(f"  {k:14s} {c:16s} {v / n:14.0f}")
PY
