# round 5, call ar: the overflow launch reading its counts beside the gate word, against HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ar}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_members_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V='{"inplace": {"INPLACE": "1"}, "copy": {}}'
for r in 1 2 3 4; do
  for v in new head; do
    L=$PWD/ringpop-node_amd/librpamd.so; [ $v != new ] && L=$PWD/ringpop-node_amd/ab/librpamd_$v.so
    RP_AMD_LIB=$L timeout -k 10 200 python -u tools/ab_fold.py --rounds 8 --out $O/${v}_$r.json --variants "$V" > $O/${v}_$r.log 2>&1 || { echo "ab $v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('$v $r', {k:(v['median_ms'],v['min_ms']) for k,v in d.items()})"
  done
done
