# round 5, call g: the service with 8 warm loads a poll (32 KB, the compact tables every ~0.15 ms), with and
# without the L2 warm loads; device phase stamps (RP_SVC_PROF); service parity tests first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "service" > gpurun_out/r05g_svc.log 2>&1 || { echo "service tests failed"; tail -40 gpurun_out/r05g_svc.log; exit 1; }
tail -2 gpurun_out/r05g_svc.log
O=gpurun_out/r05g; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" RP_SVC_PROF=1 timeout -k 10 120 node tools/svc_latency.js > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; return 1; }
  echo "$n $(cat $O/$n.json)"; grep "\[rp\] service" $O/$n.err || true
}
for rep in 1 2; do
  run v1_$rep RP_RING_SVC=1 &&
  run v3_$rep RP_RING_SVC=2 &&
  run v3w0_$rep RP_RING_SVC=2 RP_SVC_WARM=0 || exit 1
done
