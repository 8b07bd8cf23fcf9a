# round 5, call x: the hinted index built by the first batch lookupN(3) instead of every ring rebuild
# (per-call mutation cost), the direct-table service: ring GPU tests, then the node per-call API legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_ring_gpu.py tests/test_js_gpu.py tests/test_group_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
make -s -C ringpop-node_amd/js > /dev/null
timeout -k 10 300 node tools/api_latency.js > $O/api.json 2> $O/api.err || { echo api failed; tail -20 $O/api.err; exit 1; }
python3 -c "
import json; a=json.load(open('$O/api.json'))
print({k: (a[k].get('median_us_per_mutation') or a[k].get('median_us')) for k in ('lookup','lookup_service','lookupN3_service','addServer','addRemoveServers') if k in a})
"
