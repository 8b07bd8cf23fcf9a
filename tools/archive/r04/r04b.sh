# round 4, call b: ring + JS tests (service on the compact walk, single-key N-API entries), the
# per-call API latency, PMC of the kept 4,096-id bucket fold, and a full bench + kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_ring_gpu.py tests/test_js_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 node tools/api_latency.js 10000 1332 > $O/api.json 2> $O/api.err || { echo api failed; tail -20 $O/api.err; exit 1; }
cat $O/api.json
timeout -k 10 400 bash tools/pmc_bk.sh $O/pmc_bk > $O/pmc_bk.log 2>&1 || { echo pmc failed; tail -20 $O/pmc_bk.log; exit 1; }
cat $O/pmc_bk.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu --no-api > $O/bench_prof.json 2> $O/bench_prof.err || { echo prof failed; tail -20 $O/bench_prof.err; exit 1; }
echo done
