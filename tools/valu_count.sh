# SQ_INSTS_VALU per extractor kernel over tools/prof_stages.py (one PMC pass) + extractor parity
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/valu_count; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py > $O/ext.log 2>&1; rc=$?; tail -2 $O/ext.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d $O/p -o p --output-format csv -- python3 tools/prof_stages.py --frames 32 --iters 5 --mode ext > $O/p.log 2>&1 || { echo "pmc failed"; tail -3 $O/p.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/p/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: [0.0, 0])
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1].split('<')[0]
    acc[k][0] += float(r['Counter_Value']); acc[k][1] += 1
for k, (v, n) in sorted(acc.items()):
    print(f"{k:20s} dispatches {n:6d}  VALU insts per dispatch {v / n:14.0f}")
PY
