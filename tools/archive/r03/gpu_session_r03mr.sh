cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03mr
L="--sim-n 0 --sim5-n 0 --no-wire --no-api --no-cpu --steps 20 --warmup 5"
for i in 1 2 3; do for r in 300; do
timeout -k 10 300 python3 -u bench.py $L --ramp-ms $r > gpurun_out/r03mr/r$r.$i.json 2> gpurun_out/r03mr/r$r.$i.err || { echo failed; tail gpurun_out/r03mr/r$r.$i.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); m=d['merge']; print(sys.argv[1], round(d['value']/1e9,2), 'fold', round(m['fold']['ms_per_batch'],4), 'large', round(m['fold_large']['ms_per_batch'],4), 'c3', round(m['ms_per_batch'],4))" gpurun_out/r03mr/r$r.$i.json
done; done
