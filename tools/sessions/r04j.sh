# round 4, call j: wire decoder, records a lane per member (ab/librpamd_mp.so, -DRP_WIRE_MEMBERS=1)
# against the in-tree per-record walk: wire GPU tests on the mp build, wave phase cycles of
# both (wprof / wprof0), then the wire leg alternating the two libraries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j; mkdir -p $O
RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_mp.so timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/wiretest_mp.log 2>&1 || { echo wire tests failed; tail -30 $O/wiretest_mp.log; exit 1; }
tail -1 $O/wiretest_mp.log
for v in wprof0 wprof; do
RP_WIRE_DEBUG=1 RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/$v.json 2> $O/$v.err || { echo bench $v failed; tail -20 $O/$v.err; exit 1; }
echo $v; grep "wire wave cycles" $O/$v.err | tail -1; grep "by waves" $O/$v.err | tail -1
done
for i in 1 2; do
  for v in tree mp; do
    if [ $v = mp ]; then export RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_mp.so; else unset RP_AMD_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/$v$i.json 2> $O/$v$i.err || { echo "bench $v failed"; tail -20 $O/$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], 'enc', round(d['encode']['ms'],3), 'dec', round(d['decode']['ms'],3), d['round_trip_ok'])" $O/$v$i.json $v
  done
done
