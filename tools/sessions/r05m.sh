# round 5, call m: bucket fold 8-B records, in-place outputs, two tiles a lane: parity, A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_members_gpu.py -k "bucket_fold" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/ab_fold.py --rounds 8 --out $O/ab.json --variants '{"rec8": {}, "rec12": {"RP_BK_REC8": "0"}, "single": {"RP_BK_PAIR": "0"}, "pair_inplace": {"INPLACE": "1"}, "single_inplace": {"RP_BK_PAIR": "0", "INPLACE": "1"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
cat $O/ab.json
