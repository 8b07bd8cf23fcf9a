# round 6, call w: kernel times of the id-partitioned fold's per-rank share (tools/part_fold.py
# under rocprofv3 --kernel-trace --stats)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06w}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/part_fold.py --reps 6 > $O/part_fold.json 2> $O/prof.err || { echo "rocprof failed"; tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
head -12 $O/kernel_stats.csv
