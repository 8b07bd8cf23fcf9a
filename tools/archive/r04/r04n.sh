# round 4, call n: wire decoder in two passes (first pass 1,280 tokens / 10 waves a CU, the rest in
# the full layout) against the full layout alone (RP_WIRE_ONEPASS=1, same library): wire + JS GPU
# tests, then alternating wire legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py tests/test_js_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/wiretest.log 2>&1 || { echo wire tests failed; tail -30 $O/wiretest.log; exit 1; }
tail -1 $O/wiretest.log
for i in 1 2; do
  for v in onepass twopass; do
    if [ $v = onepass ]; then export RP_WIRE_ONEPASS=1; else unset RP_WIRE_ONEPASS; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/$v$i.json 2> $O/$v$i.err || { echo "bench $v failed"; tail -20 $O/$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], 'enc', round(d['encode']['ms'],3), 'dec', round(d['decode']['ms'],3), d['round_trip_ok'])" $O/$v$i.json $v
  done
done
