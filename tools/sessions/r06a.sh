# round 6, call a: the full GPU suite with the process-wide service quiesce (QuietScope), the
# status range checks and the new service-beside-membership test; then the default bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06a}; mkdir -p $O
timeout -k 10 180 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_ring_gpu.py -k "service" > $O/svc.log 2>&1 || { echo "svc tests failed"; tail -40 $O/svc.log; exit 1; }
tail -1 $O/svc.log
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
