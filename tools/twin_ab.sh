set -e
timeout -k 10 400 python -u -m pytest tests/test_sim_gpu.py tests/test_sim_shard_gpu.py tests/test_sim_digests_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/tw_tests.log 2>&1
for tw in 1 0; do
  RP_SIM_TWINS=$tw timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-merge --no-wire --sim5-cpu 0 > gpurun_out/tw_$tw.json 2> gpurun_out/tw_$tw.err
done
