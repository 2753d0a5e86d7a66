# rocprofv3 kernel stats of the LBA (C4) and LocalInertialBA side lines (one gpurun call)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/lba_stats; rm -rf $O; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/lba -o lba -- python3 tools/bench_lba.py --calls 20 --cpu-calls 0 > $O/lba.json 2> $O/lba.err || { echo "lba failed"; tail -3 $O/lba.err; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/lia -o lia -- python3 tools/bench_lba.py --lia --calls 20 --cpu-calls 0 > $O/lia.json 2> $O/lia.err || { echo "lia failed"; tail -3 $O/lia.err; exit 1; }
cp $(find $O/lba -name '*kernel_stats.csv' | head -n1) $O/lba_kernel_stats.csv
cp $(find $O/lia -name '*kernel_stats.csv' | head -n1) $O/lia_kernel_stats.csv
tail -c 300 $O/lba.json; echo; tail -c 300 $O/lia.json
