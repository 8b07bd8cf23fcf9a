# round 6, call ab: k_ck_lanes fixup statistics per refresh over the C5 run (-DRP_CKL_STAT build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ab}; mkdir -p $O
RP_AMD_LIB=$GRAFT_REPO_ROOT/ringpop-node_amd/librpamd_ckl.so RP_CKL_STAT_PRINT=1 timeout -k 10 300 python3 -u tools/c5_rounds.py --label ckl > $O/c5_ckl.json 2> $O/c5_ckl.err || { echo "c5 failed"; tail $O/c5_ckl.err; exit 1; }
grep "k_ck_lanes" $O/c5_ckl.err | head -60
