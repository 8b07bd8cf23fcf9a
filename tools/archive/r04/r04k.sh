# round 4, call k: wire decoder with the records' names looked up together by default and the
# record stash kept in the handle's scratch (in-tree) against ab/librpamd_split.so (same kernels,
# stash allocated per call): wire + JS GPU tests, phase cycles, alternating wire legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k; mkdir -p $O
A=$PWD/ringpop-node_amd/ab
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py tests/test_js_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/wiretest.log 2>&1 || { echo wire tests failed; tail -30 $O/wiretest.log; exit 1; }
tail -1 $O/wiretest.log
RP_AMD_LIB=$A/librpamd_wprof.so timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/wprof.json 2> $O/wprof.err || { echo bench wprof failed; tail -20 $O/wprof.err; exit 1; }
grep "wire wave cycles" $O/wprof.err | tail -1
for i in 1 2; do
  for v in split tree; do
    if [ $v = tree ]; then unset RP_AMD_LIB; else export RP_AMD_LIB=$A/librpamd_$v.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/$v$i.json 2> $O/$v$i.err || { echo "bench $v failed"; tail -20 $O/$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], 'enc', round(d['encode']['ms'],3), 'dec', round(d['decode']['ms'],3), d['round_trip_ok'])" $O/$v$i.json $v
  done
done
