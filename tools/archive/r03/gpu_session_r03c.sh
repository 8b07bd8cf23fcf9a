mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_members_gpu.py tests/test_prims_gpu.py tests/test_merge_shard_gpu.py > gpurun_out/t6.log 2>&1; echo "tests rc=$?"; tail -15 gpurun_out/t6.log
timeout -k 10 300 python3 tools/merge_fold_ab.py > gpurun_out/ab_part.json 2>gpurun_out/ab_part.err; echo "ab rc=$?"; cat gpurun_out/ab_part.json
RP_MEMBERS_PART=0 timeout -k 10 300 python3 tools/merge_fold_ab.py --only big > gpurun_out/ab_nopart.json 2>gpurun_out/ab_nopart.err; echo "ab0 rc=$?"; cat gpurun_out/ab_nopart.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_part -o run -- python3 tools/merge_fold_ab.py --reps 10 > gpurun_out/prof_part.log 2>&1; echo "prof rc=$?"
for e in 0 1; do RP_SIM_EARLY=$e timeout -k 10 300 python3 bench.py --no-merge --no-wire --no-cpu --no-api --steps 2 --warmup 1 --batch-log2 20 > gpurun_out/sim_early$e.json 2> gpurun_out/sim_early$e.err; echo "sim early=$e rc=$?"; done
