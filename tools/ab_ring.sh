# A/B of the C2 lookup leg: the in-tree librpamd.so against ab/librpamd_base.so, alternating,
# after the ring GPU tests on the in-tree build. Usage (GPU box): bash tools/ab_ring.sh TAG
set -u
cd $GRAFT_REPO_ROOT
tag=${1:-abr}
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_ring_gpu.py tests/test_group_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$tag/ringtest.log 2>&1 || { echo "ring tests failed"; tail -30 gpurun_out/$tag/ringtest.log; exit 1; }
tail -1 gpurun_out/$tag/ringtest.log
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export RP_AMD_LIB=$PWD/tools/ablib/librpamd_base.so; else unset RP_AMD_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu --sim-n 0 --sim5-n 0 --no-merge --no-wire --no-api --steps 20 --warmup 5 > gpurun_out/$tag/$v$i.json 2> gpurun_out/$tag/$v$i.err || { echo "bench $v failed"; tail -20 gpurun_out/$tag/$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],4), 'ms/step', 'op', round(d['roofline']['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))" gpurun_out/$tag/$v$i.json $v
  done
done
