# round 5, call f: the single-wave host-hashed service (k_lookup_service3) against the round-4 kernel, with and
# without the L2 warm loads; device phase stamps (RP_SVC_PROF); service parity tests first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "service" > gpurun_out/r05f_svc.log 2>&1 || { echo "service tests failed"; tail -40 gpurun_out/r05f_svc.log; exit 1; }
tail -2 gpurun_out/r05f_svc.log
O=gpurun_out/r05f; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" RP_SVC_PROF=1 timeout -k 10 120 node tools/svc_latency.js > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; return 1; }
  echo "$n $(cat $O/$n.json)"; grep "\[rp\] service" $O/$n.err || true
}
for rep in 1 2 3; do
  run v1_$rep RP_RING_SVC=1 &&
  run v3_$rep RP_RING_SVC=2 &&
  run v3w0_$rep RP_RING_SVC=2 RP_SVC_WARM=0 || exit 1
done
# the bucket fold's direct applied stores (RP_BK_DIRECT) against the map + gather
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_members_gpu.py > $O/members.log 2>&1 || { echo "members tests failed"; tail -40 $O/members.log; exit 1; }
tail -2 $O/members.log
timeout -k 10 300 python -u tools/ab_fold.py --rounds 10 --out $O/ab_fold.json --variants '{"direct": {}, "gather": {"RP_BK_DIRECT": "0"}}' > $O/ab_fold.log 2>&1 || { echo "ab failed"; tail -30 $O/ab_fold.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_fold.json'))
for k,v in d.items(): print(k, v['median_ms'], v['min_ms'], v['frac_49B'])"
