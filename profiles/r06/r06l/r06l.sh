# round 6, call l: the 2^22 bucket fold's per-workgroup timeline (diagnostics build, -DRP_BK_PROF)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06l}; mkdir -p $O
RP_AMD_LIB=$GRAFT_REPO_ROOT/ringpop-node_amd/librpamd_bkprof.so RP_BK_PROF_PRINT=1 timeout -k 10 300 python3 -u tools/merge_fold_ab.py --only big --inplace --reps 6 > $O/bkprof.json 2> $O/bkprof.err || { echo "failed"; tail -20 $O/bkprof.err; exit 1; }
grep "k_bk_fold" $O/bkprof.err | tail -8
cat $O/bkprof.json
