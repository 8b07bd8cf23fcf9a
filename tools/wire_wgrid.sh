# encoder grid sweep (k_rec_write_lds workgroups, RP_WIRE_WGRID), after the wire GPU tests
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wwg
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wwg/t.log 2>&1 || { tail -20 gpurun_out/wwg/t.log; exit 1; }
tail -1 gpurun_out/wwg/t.log
for i in 1 2; do for g in 2048 4096 8192 16384 100000; do
  RP_WIRE_WGRID=$g timeout -k 10 200 python -u bench.py --no-cpu --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > gpurun_out/wwg/g$g.$i.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], 'enc', round(d['encode']['ms'],3), 'dec', round(d['decode']['ms'],3), d['round_trip_ok'])" gpurun_out/wwg/g$g.$i.json $g
done; done
