# round 5, call d: the three-wave lookup service (RP_RING_SVC=2) vs the round-4 kernel: service
# parity tests, then the node per-call latency leg with each kernel; and the fold A/B (r05c)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "service" > $O/svc.log 2>&1 || { echo "service tests failed"; tail -40 $O/svc.log; exit 1; }
tail -2 $O/svc.log
for v in 2 1 2 1; do
  RP_RING_SVC=$v timeout -k 10 200 node tools/api_latency.js > $O/api_v$v.json 2> $O/api_v$v.err || { echo "api $v failed"; tail -5 $O/api_v$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('$O/api_v$v.json') if l.startswith('{')][-1])
print('svc v$v', 'lookup_service', d['lookup_service'], 'lookupN3_service', d['lookupN3_service'], 'lookup', d['lookup']['median_us'])"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_members_gpu.py > $O/members.log 2>&1 || { echo "members tests failed"; tail -40 $O/members.log; exit 1; }
tail -2 $O/members.log
timeout -k 10 300 python -u tools/ab_fold.py --rounds 8 --out $O/ab_fold.json --variants '{"new": {}, "old": {"RP_BK_PRE": "0", "RP_BK_GV": "4"}, "pre-gv4": {"RP_BK_GV": "4"}, "pre0-gv16": {"RP_BK_PRE": "0"}}' > $O/ab_fold.log 2>&1 || { echo "ab failed"; tail -30 $O/ab_fold.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_fold.json'))
for k,v in d.items(): print(k, v['median_ms'], v['min_ms'], v['frac_49B'])"
