# round 4, call zj (end of round, final code): the whole GPU suite, smoke(), the
# default bench.py line, and rocprofv3 kernel stats of the same bench command
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04zj; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu --no-api > $O/bench_prof.json 2> $O/bench_prof.err || { echo prof failed; tail -20 $O/bench_prof.err; exit 1; }
echo done
