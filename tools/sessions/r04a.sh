# round 4, call a: the advisor fixes' GPU tests (merge shards, JS drop-ins, ring, members), then
# the lean lookup kernel's phase counters on C2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_merge_shard_gpu.py tests/test_js_gpu.py tests/test_ring_gpu.py tests/test_members_gpu.py tests/test_sim_shard_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
RP_AMD_LIB=ringpop-node_amd/librpamd_lkprof.so RP_LK_PROF_PRINT=1 timeout -k 10 200 python3 -u tools/lk_phase.py > $O/lk_phase.log 2>&1 || { echo lk_phase failed; tail -20 $O/lk_phase.log; exit 1; }
tail -12 $O/lk_phase.log
RP_LOOKUP_STG=1 RP_AMD_LIB=ringpop-node_amd/librpamd_lkprof.so RP_LK_PROF_PRINT=1 LK_LAUNCHES=30 timeout -k 10 200 python3 -u tools/lk_phase.py > $O/lk_phase_stg1.log 2>&1 || { echo lk_phase stg1 failed; tail -20 $O/lk_phase_stg1.log; exit 1; }
tail -6 $O/lk_phase_stg1.log
timeout -k 10 300 node tools/api_latency.js 10000 1332 > $O/api.json 2> $O/api.err || { echo api failed; tail -20 $O/api.err; exit 1; }
cat $O/api.json
