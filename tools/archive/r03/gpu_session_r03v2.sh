cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03v2
L="--no-merge --sim-n 0 --sim5-n 0 --no-wire --no-api --no-cpu --steps 20 --warmup 5"
timeout -k 10 200 python3 -u bench.py $L --ramp-ms 0 > gpurun_out/r03v2/ramp0.json 2> gpurun_out/r03v2/ramp0.err || { echo r0 failed; tail gpurun_out/r03v2/ramp0.err; exit 1; }
timeout -k 10 200 python3 -u bench.py $L > gpurun_out/r03v2/ramp300.json 2> gpurun_out/r03v2/ramp300.err || { echo r300 failed; tail gpurun_out/r03v2/ramp300.err; exit 1; }
timeout -k 10 200 python3 -u bench.py $L --ramp-ms 1000 > gpurun_out/r03v2/ramp1000.json 2> gpurun_out/r03v2/ramp1000.err || { echo r1000 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03v2/prof -o run -- python3 -u bench.py $L --ramp-ms 1000 > gpurun_out/r03v2/prof.json 2> gpurun_out/r03v2/prof.err || { echo prof failed; tail gpurun_out/r03v2/prof.err; exit 1; }
for f in ramp0 ramp300 ramp1000 prof; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/r03v2/$f.json').read().strip().splitlines()[-1]); print('$f', d['value']/1e9, d['ms_per_step'], d['warmup_ramp_steps'], d['roofline']['kernel_ms'])"; done
