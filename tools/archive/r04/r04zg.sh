# round 4, call zg: the lookup service's host side skips the stream query while the wave is known
# to be polling (in-tree) against the previous commit (ab/hd/librpamd.so through LD_LIBRARY_PATH,
# the addon's RUNPATH); ring tests incl. the service, then the per-call latency leg alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04zg; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "service or small_host" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in head tree; do
    if [ $v = head ]; then export LD_LIBRARY_PATH=$PWD/ringpop-node_amd/ab/hd; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 300 node tools/api_latency.js 10000 1332 > $O/api_$v$i.json 2> $O/api_$v$i.err || { echo api failed; tail -20 $O/api_$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], 'svc', round(d['lookup_service']['median_us'],2), 'svcN', round(d['lookupN3_service']['median_us'],2), 'launch', round(d['lookup']['median_us'],2))" $O/api_$v$i.json $v
  done
done
