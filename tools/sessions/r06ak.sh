# round 6, call ak: range updates with the rank's changes packed first (k_part_*): parity (merge
# shard + members suites), then one rank's share of the 2^22 fold per G, packed against unpacked
# (RP_BK_PART_PACK=0), alternating processes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ak}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_merge_shard_gpu.py tests/test_members_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 1 0; do
    RP_BK_PART_PACK=$v timeout -k 10 300 python3 -u tools/part_fold.py --reps 12 > $O/part_pack${v}_$rep.json 2> $O/part_pack${v}_$rep.err || { echo "part_fold failed $v"; tail -20 $O/part_pack${v}_$rep.err; exit 1; }
    echo "pack=$v rep=$rep $(cat $O/part_pack${v}_$rep.json)"
  done
done
