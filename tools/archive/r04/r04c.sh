# round 4, call c: 12-B bucket records + 2-bit result map: members tests, fold A/B against the
# round-3 record layout (ringpop-node_amd/ab/librpamd_base.so), PMC of the new layout
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py tests/test_damp_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  for lib in ringpop-node_amd/ab/librpamd_base.so ringpop-node_amd/librpamd.so; do
    RP_AMD_LIB=$lib timeout -k 10 200 python3 -u tools/merge_fold_ab.py --only big --reps 20 >> $O/fold_ab.jsonl 2>> $O/fold_ab.err || { echo fold ab failed; tail -20 $O/fold_ab.err; exit 1; }
  done
done
cat $O/fold_ab.jsonl
timeout -k 10 400 bash tools/pmc_bk.sh $O/pmc_bk > $O/pmc_bk.log 2>&1 || { echo pmc failed; tail -20 $O/pmc_bk.log; exit 1; }
cat $O/pmc_bk.log
