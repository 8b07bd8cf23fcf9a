# round 6, call ar: PMC retakes: the 2^22 bucket fold in place (bytes, L2 write requests, SQ wait
# share; tools/pmc_bk.sh) and the C5 refresh kernels over the first 12 rounds with the sorted
# order (default) and list order (RP_SIM_CK_SORT=0) (tools/pmc_ck.sh); separate --pmc passes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ar}; mkdir -p $O
PMC_BK_ARGS="--inplace" bash tools/pmc_bk.sh $O/pmc_bk > $O/pmc_bk.out 2>&1 || { echo "pmc_bk failed"; tail -20 $O/pmc_bk.out; exit 1; }
cat $O/pmc_bk.out
python3 tools/pmc_merge_summary.py $O/pmc_bk > $O/pmc_bk_summary.json || { echo "summary failed"; exit 1; }
bash tools/pmc_ck.sh $O/pmc_ck_sorted 12 > $O/pmc_ck_sorted.out 2>&1 || { echo "pmc_ck failed"; tail -20 $O/pmc_ck_sorted.out; exit 1; }
cat $O/pmc_ck_sorted.out
RP_SIM_CK_SORT=0 bash tools/pmc_ck.sh $O/pmc_ck_list 12 > $O/pmc_ck_list.out 2>&1 || { echo "pmc_ck list failed"; tail -20 $O/pmc_ck_list.out; exit 1; }
cat $O/pmc_ck_list.out
