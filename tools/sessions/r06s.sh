# round 6, call s: the service's idle waves touching their slice of the direct table
# (RP_SVC_WARM=2, loads issued before each poll) against no touching, cold keys (8,192 distinct), then hot (16)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06s}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ring_gpu.py -k "service" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in 0:8192 2:8192 0:16; do
    a=${v%:*}; k=${v#*:}
    RP_SVC_WARM=$a timeout -k 10 120 node tools/svc_latency.js 10000 4000 $k > $O/lat_${a}_${k}_$rep.json 2> $O/lat_${a}_${k}_$rep.err || { echo "latency run failed $v"; cat $O/lat_${a}_${k}_$rep.err; exit 1; }
    echo "warm=$a keys=$k rep=$rep $(python3 -c "import json,sys;d=json.load(open('$O/lat_${a}_${k}_$rep.json'));print(d['lookup_service']['median_us'],d['lookup_service']['p10_us'],d['lookup_service']['p90_us'],d['lookupN3_service']['median_us'],d['lookupN3_service']['p90_us'])")"
  done
done
