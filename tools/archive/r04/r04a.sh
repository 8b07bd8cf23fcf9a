# round 4, call a: the advisor fixes' GPU tests (merge shards, JS drop-ins, ring incl. the new
# lookup variants and the service, members, sim shards, bench), the lean kernel's phase counters
# on C2, the staging / halves A/B, and the per-call API latency
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_ring_gpu.py tests/test_merge_shard_gpu.py tests/test_js_gpu.py tests/test_members_gpu.py tests/test_sim_shard_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u tools/ab_lookup.py --rounds 6 --only default/lookupN3,stg1/lookupN3,lh2/lookupN3,stg2/lookupN3,stg2-lh1/lookupN3,stg2-hs4/lookupN3 > $O/ab.json 2> $O/ab.err || { echo ab failed; tail -20 $O/ab.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/ab.json'));[print(k, round(v['median_ms'],4), round(v['min_ms'],4), v['digest']) for k,v in d.items()]"
for v in 0 2; do
RP_LOOKUP_STG=$v RP_AMD_LIB=ringpop-node_amd/librpamd_lkprof.so RP_LK_PROF_PRINT=1 LK_LAUNCHES=30 timeout -k 10 200 python3 -u tools/lk_phase.py > $O/lk_phase_stg$v.log 2>&1 || { echo lk_phase failed; tail -20 $O/lk_phase_stg$v.log; exit 1; }
tail -4 $O/lk_phase_stg$v.log
done
timeout -k 10 300 node tools/api_latency.js 10000 1332 > $O/api.json 2> $O/api.err || { echo api failed; tail -20 $O/api.err; exit 1; }
cat $O/api.json
