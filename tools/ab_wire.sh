# A/B of the wire leg: the in-tree librpamd.so against ringpop-node_amd/ab/librpamd_base.so, alternating, plus
# the wire GPU tests on the in-tree build. Usage (on the GPU box): bash tools/ab_wire.sh TAG
set -u
cd $GRAFT_REPO_ROOT
tag=${1:-ab}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/wiretest.log 2>&1 || { echo "wire tests failed"; tail -30 gpurun_out/$tag/wiretest.log; exit 1; }
tail -1 gpurun_out/$tag/wiretest.log
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_base.so; else unset RP_AMD_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > gpurun_out/$tag/$v$i.json 2> gpurun_out/$tag/$v$i.err || { echo "bench $v failed"; tail -20 gpurun_out/$tag/$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], 'enc', round(d['encode']['ms'],3), 'dec', round(d['decode']['ms'],3), d['round_trip_ok'])" gpurun_out/$tag/$v$i.json $v
  done
done
