# round 4, call f: how often k_ck_lanes' waves run a piece fixup at C5 (-DRP_CKL_STAT build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f; mkdir -p $O
RP_AMD_LIB=ringpop-node_amd/librpamd_cklstat.so RP_CKL_STAT_PRINT=1 timeout -k 10 400 python3 -u tools/sim_c5_probe.py 100000 36 > $O/c5_stat.log 2>&1 || { echo probe failed; tail -20 $O/c5_stat.log; exit 1; }
cat $O/c5_stat.log
