# round 6, call u: the partitioned merge (PartMembership, rp_members_update_range_dev) GPU tests
# and the members suite; then the node latency tools side by side (api_latency.js as bench.py
# runs it, svc_latency.js), alternating, to compare the two service figures on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06u}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_merge_shard_gpu.py tests/test_members_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 node tools/api_latency.js > $O/api_$rep.json 2> $O/api_$rep.err || { echo "api failed"; tail $O/api_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/api_$rep.json'));print('api', d['lookup_service']['median_us'], d['lookupN3_service']['median_us'])"
  timeout -k 10 120 node tools/svc_latency.js 10000 2000 8192 > $O/svc_$rep.json 2> $O/svc_$rep.err || { echo "svc failed"; tail $O/svc_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/svc_$rep.json'));print('svc', d['lookup_service']['median_us'], d['lookupN3_service']['median_us'])"
done
