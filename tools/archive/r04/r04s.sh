# round 4, call s: the grouped fold's k_link + k_fold_fast in one launch with a grid barrier
# (k_link_fold, in-tree default) against the two launches (RP_MEMBERS_FUSE=0, same library):
# members / merge-shard / JS GPU tests, then alternating C3 merge legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py tests/test_js_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in two fused; do
    if [ $v = two ]; then export RP_MEMBERS_FUSE=0; else unset RP_MEMBERS_FUSE; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu --no-api --no-wire --sim-n 0 --sim5-n 0 --steps 2 --warmup 1 --batch-log2 20 > $O/$v$i.json 2> $O/$v$i.err || { echo "bench $v failed"; tail -20 $O/$v$i.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['merge']
f=d.get('fold',{}); fl=d.get('fold_large',{})
print(sys.argv[2], 'batch_us', round(d['ms_per_batch']*1e3,2), 'fold_ms', f.get('ms_per_batch'), 'large_ms', fl.get('ms_per_batch'))" $O/$v$i.json $v
  done
done
