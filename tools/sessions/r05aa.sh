# round 5, call aa: 8-B member rows (incarnation << 3 | exists << 2 | status) with the grouped fold's
# counters in their own array: membership GPU tests, then the 2^22 fold A/B against the previous
# commit's library (ab/librpamd_rows16.so), alternating processes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py tests/test_damp_gpu.py tests/test_js_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
V='{"copy": {}, "inplace": {"INPLACE": "1"}}'
for r in 1 2; do
  timeout -k 10 200 python -u tools/ab_fold.py --rounds 8 --out $O/new$r.json --variants "$V" > $O/new$r.log 2>&1 || { echo "ab new failed"; tail -20 $O/new$r.log; exit 1; }
  RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_rows16.so timeout -k 10 200 python -u tools/ab_fold.py --rounds 8 --out $O/old$r.json --variants "$V" > $O/old$r.log 2>&1 || { echo "ab old failed"; tail -20 $O/old$r.log; exit 1; }
done
for f in new1 old1 new2 old2; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', {k:(v['median_ms'],v['min_ms']) for k,v in d.items()})"; done
timeout -k 10 300 python3 -u tools/merge_fold_ab.py --only c3,c3ck --reps 20 > $O/c3_new.json 2> $O/c3_new.err || { echo c3 failed; tail $O/c3_new.err; exit 1; }
RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_rows16.so timeout -k 10 300 python3 -u tools/merge_fold_ab.py --only c3,c3ck --reps 20 > $O/c3_old.json 2> $O/c3_old.err || { echo c3 old failed; tail $O/c3_old.err; exit 1; }
python3 -c "
import json
for f in ('c3_new','c3_old'):
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, {k:(round(d[k]['ms_mean'],4), round(d[k]['ms_p50'],4)) for k in ('c3','c3ck')})"
