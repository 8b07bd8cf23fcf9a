cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03v1
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ > gpurun_out/r03v1/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03v1/tests.log; exit 1; }
tail -2 gpurun_out/r03v1/tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v1/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r03v1/smoke.log; exit 1; }
cat gpurun_out/r03v1/smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03v1/bench.json 2> gpurun_out/r03v1/bench.err || { echo bench failed; tail -20 gpurun_out/r03v1/bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03v1/prof -o run -- python3 -u bench.py --no-cpu --no-api > gpurun_out/r03v1/bench_prof.json 2> gpurun_out/r03v1/bench_prof.err || { echo prof failed; tail -20 gpurun_out/r03v1/bench_prof.err; exit 1; }
echo done
