# round 6, call i: the chain kernels alone (no folds beside them): packed vs one workgroup a string
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06i}; mkdir -p $O
timeout -k 10 300 python3 -u tools/hl_bench.py --n 16,128,256,512 --reps 2 > $O/hl.log 2>&1 || { echo "hl failed"; tail -20 $O/hl.log; exit 1; }
grep -v "^{" $O/hl.log
