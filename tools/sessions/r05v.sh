# round 5, call v: the default bench.py line and rocprofv3 --kernel-trace --stats of the same bench (CPU legs off)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05v}; mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --no-cpu --no-api > $O/bench_prof.json 2> $O/bench_prof.err || { echo prof failed; tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/bench_kernel_stats.csv; rm -rf $O/prof
head -6 $O/bench_kernel_stats.csv | cut -c1-200
