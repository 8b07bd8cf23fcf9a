# round 6, call m: the lookup service with several independent pollers (RP_SVC_WAVES) — parity,
# then per-call latency alternating 1 / 2 / 4 / 8 waves in node on the C2 ring
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06m}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ring_gpu.py -k "service" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2; do
  for w in 1 8 2 4; do
    RP_SVC_WAVES=$w timeout -k 10 120 node tools/svc_latency.js 10000 4000 > $O/lat_w${w}_$rep.json 2> $O/lat_w${w}_$rep.err || { echo "latency run failed w=$w"; cat $O/lat_w${w}_$rep.err; exit 1; }
    echo "w=$w rep=$rep $(cat $O/lat_w${w}_$rep.json)"
  done
done
