# round 5, call e: lookup service phase breakdown (RP_SVC_PROF) and knobs: the round-4 kernel
# against the three-wave one at 8 / 4 / 1 polls in flight, with and without the L2 warm wave
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
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
