# round 5, call w: the service's direct table (one 64-B record per key, k_dt_build): service parity
# tests, then the node single-call latency with and without it (RP_SVC_DT=0) and the device stamps
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "service" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
make -s -C ringpop-node_amd/js > /dev/null
for r in 1 2 3; do
  for v in dt win; do
    if [ $v = win ]; then export RP_SVC_DT=0; else unset RP_SVC_DT; fi
    RP_SVC_PROF=1 timeout -k 10 120 node tools/svc_latency.js > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    echo "$v $r $(cat $O/${v}_$r.json | head -c 300)"; grep "service:" $O/${v}_$r.err | tail -1
  done
done
