# round 6, call f: is the C3 stream host-bound? host enqueue time per batch, and a kernel trace
# of a 256-batch C3 stream (side build on) for the GPU-side gaps
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06f}; mkdir -p $O
timeout -k 10 300 python3 -u tools/c3_host.py --batches 256 > $O/c3host.log 2>&1 || { echo "c3host failed"; tail -20 $O/c3host.log; exit 1; }
grep -v "^{" $O/c3host.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python3 -u tools/c3_ab.py --batches 256 --rounds 1 --variants side > $O/c3prof.log 2>&1 || { echo "prof failed"; tail -20 $O/c3prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
