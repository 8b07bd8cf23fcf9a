mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_merge_shard_gpu.py tests/test_js_gpu.py tests/test_members_gpu.py tests/test_sim_gpu.py tests/test_sim_shard_gpu.py tests/test_sim_digests_gpu.py tests/test_bench_gpu.py > gpurun_out/t5.log 2>&1
echo "tests rc=$?"; tail -4 gpurun_out/t5.log
timeout -k 10 300 node tools/api_latency.js > gpurun_out/api.json 2> gpurun_out/api.err; echo "api rc=$?"
for e in 0 1; do RP_SIM_EARLY=$e timeout -k 10 300 python3 bench.py --no-merge --no-wire --no-cpu --no-api --steps 2 --warmup 1 --batch-log2 20 > gpurun_out/sim_early$e.json 2> gpurun_out/sim_early$e.err; echo "sim early=$e rc=$?"; done
timeout -k 10 300 python3 tools/ab_lookup.py --rounds 7 --only default/lookupN3,occ5/lookupN3,probe/ablate-hash-only > gpurun_out/ab_occ.json 2>&1; echo "ab rc=$?"
