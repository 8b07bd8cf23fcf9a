# round 5, call ap: the fold's records walk with both of a lane's segments (and their first 6
# records) in flight together, the overflow gate read beside the counts: members tests, then 2^22
# A/B against ab/librpamd_head.so (HEAD) and ab/librpamd_p4.so (4 records up front)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ap}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_members_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V='{"inplace": {"INPLACE": "1"}, "copy": {}}'
for r in 1 2 3; do
  for v in new head p4; do
    L=$PWD/ringpop-node_amd/librpamd.so; [ $v != new ] && L=$PWD/ringpop-node_amd/ab/librpamd_$v.so
    RP_AMD_LIB=$L timeout -k 10 200 python -u tools/ab_fold.py --rounds 8 --out $O/${v}_$r.json --variants "$V" > $O/${v}_$r.log 2>&1 || { echo "ab $v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('$v $r', {k:(v['median_ms'],v['min_ms']) for k,v in d.items()})"
  done
done
