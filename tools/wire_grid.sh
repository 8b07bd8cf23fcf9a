cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wg
for i in 1 2; do for g in 512 1024 2048 8192 25000; do
  RP_WIRE_GRID=$g timeout -k 10 200 python -u bench.py --no-cpu --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > gpurun_out/wg/g$g.$i.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], round(d['decode']['ms'],3), d['round_trip_ok'])" gpurun_out/wg/g$g.$i.json $g
done; done
