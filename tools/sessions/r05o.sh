# round 5, call o: bucket fold at 52 KB of LDS (first change by CAS, no count array, 256-entry
# repeated list; three workgroups per CU) vs the committed fold (ab/librpamd_fold0.so): parity, A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
V='{"copy": {}, "inplace": {"INPLACE": "1"}}'
for r in 1 2; do
  timeout -k 10 200 python -u tools/ab_fold.py --rounds 8 --out $O/new$r.json --variants "$V" > $O/new$r.log 2>&1 || { echo "ab new failed"; tail -20 $O/new$r.log; exit 1; }
  RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_fold0.so timeout -k 10 200 python -u tools/ab_fold.py --rounds 8 --out $O/old$r.json --variants "$V" > $O/old$r.log 2>&1 || { echo "ab old failed"; tail -20 $O/old$r.log; exit 1; }
done
for f in new1 old1 new2 old2; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', {k:(v['median_ms'],v['min_ms']) for k,v in d.items()})"; done
