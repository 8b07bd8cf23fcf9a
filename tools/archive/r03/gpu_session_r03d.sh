mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/t7.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t7.log
tools/pmc_merge.sh gpurun_out/pmc_merge_r03 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err; echo "bench rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r03a -o run -- python3 bench.py --no-cpu --no-api > gpurun_out/bench_r03a_prof.json 2> gpurun_out/bench_r03a_prof.err; echo "prof rc=$?"
