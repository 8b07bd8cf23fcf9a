# round 6, call an: the service's slice table (RP_SVC_DT2=1: 32 waves, each XCD's four answering
# the requests of their eighth of a 16-MB table of 32-B records kept warm in their L2): parity,
# then node latency against the default, alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06an}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ring_gpu.py -k "service" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    RP_SVC_DT2=$v timeout -k 10 120 node tools/svc_latency.js 10000 4000 8192 > $O/lat_dt2${v}_$rep.json 2> $O/lat_dt2${v}_$rep.err || { echo "latency failed $v"; cat $O/lat_dt2${v}_$rep.err; exit 1; }
    echo "dt2=$v rep=$rep $(python3 -c "import json;d=json.load(open('$O/lat_dt2${v}_$rep.json'));print(d['lookup_service']['median_us'],d['lookup_service']['p10_us'],d['lookup_service']['p90_us'],d['lookupN3_service']['median_us'],d['lookupN3_service']['p90_us'])")"
  done
done
RP_SVC_DT2=1 RP_SVC_PROF=1 RP_SVC_WAVES=32 timeout -k 10 120 node tools/svc_latency.js 10000 4000 8192 > $O/prof_dt2.json 2> $O/prof_dt2.err || { echo "prof failed"; cat $O/prof_dt2.err; exit 1; }
cat $O/prof_dt2.err
