cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03rep
for i in 1 2 3; do
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03rep/bench$i.json 2> gpurun_out/r03rep/bench$i.err || { echo bench failed; tail -20 gpurun_out/r03rep/bench$i.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); m=d['merge']; print(sys.argv[1], round(d['value']/1e9,2), round(d['ms_per_step'],4), round(d['roofline']['frac'],4), 'c3', round(m['updates_per_s']/1e9,3), 'fold', round(m['fold']['ms_per_batch'],4), 'c5', round(d['sim_c5']['ms_per_round'],2), round(d['sim_c5']['round_ms']['p95'],1))" gpurun_out/r03rep/bench$i.json
done
