# round 6, call n: the lookup service's pollers on a staggered schedule (RP_SVC_WAVES / RP_SVC_PERIOD):
# parity, then per-call latency in node on the C2 ring, variants alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06n}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ring_gpu.py -k "service" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in 1:120 8:120 4:120 8:60 16:120 8:240; do
    w=${v%:*}; p=${v#*:}
    RP_SVC_WAVES=$w RP_SVC_PERIOD=$p timeout -k 10 120 node tools/svc_latency.js 10000 4000 > $O/lat_${w}_${p}_$rep.json 2> $O/lat_${w}_${p}_$rep.err || { echo "latency run failed $v"; cat $O/lat_${w}_${p}_$rep.err; exit 1; }
    echo "w=$w p=$p rep=$rep $(python3 -c "import json,sys;d=json.load(open('$O/lat_${w}_${p}_$rep.json'));print(d['lookup_service']['median_us'],d['lookup_service']['p90_us'],d['lookupN3_service']['median_us'],d['lookupN3_service']['p90_us'])")"
  done
done
