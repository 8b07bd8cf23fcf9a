# round 4, call j: wire decoder. In-tree: keys, values and names read as aligned dwords
# (v_alignbyte) instead of bytes; ab/librpamd_mp.so: the same plus records a lane per member;
# ab/librpamd_base.so: the previous commit. Wire GPU tests on both new builds, wave phase cycles
# (wprof0 = before, wprof = dwords); ab/librpamd_split.so: dwords + the records' address and
# source names looked up together, a name per lane, then the wire leg alternating the three libraries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j; mkdir -p $O
A=$PWD/ringpop-node_amd/ab
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py tests/test_js_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/wiretest.log 2>&1 || { echo wire tests failed; tail -30 $O/wiretest.log; exit 1; }
tail -1 $O/wiretest.log
for v in mp split; do
RP_AMD_LIB=$A/librpamd_$v.so timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/wiretest_$v.log 2>&1 || { echo $v wire tests failed; tail -30 $O/wiretest_$v.log; exit 1; }
tail -1 $O/wiretest_$v.log
done
for v in wprof0 wprof; do
RP_WIRE_DEBUG=1 RP_AMD_LIB=$A/librpamd_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/$v.json 2> $O/$v.err || { echo bench $v failed; tail -20 $O/$v.err; exit 1; }
echo $v; grep "wire wave cycles" $O/$v.err | tail -1
done
RP_WIRE_DEBUG=1 RP_AMD_LIB=$A/librpamd_mp.so timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 1 --warmup 0 --batch-log2 20 > $O/mpdbg.json 2> $O/mpdbg.err || { echo bench mpdbg failed; tail -20 $O/mpdbg.err; exit 1; }
grep "by waves" $O/mpdbg.err | tail -1
for i in 1 2; do
  for v in base tree mp split; do
    if [ $v = tree ]; then unset RP_AMD_LIB; else export RP_AMD_LIB=$A/librpamd_$v.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/$v$i.json 2> $O/$v$i.err || { echo "bench $v failed"; tail -20 $O/$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], 'enc', round(d['encode']['ms'],3), 'dec', round(d['decode']['ms'],3), d['round_trip_ok'])" $O/$v$i.json $v
  done
done
