# Sweep an environment knob over the C2 lookup leg (ramped, lookup only), two passes.
# Usage (GPU box): bash tools/sweep_env.sh TAG VAR V1 V2 ...
set -u
cd $GRAFT_REPO_ROOT
tag=$1; var=$2; shift 2
mkdir -p gpurun_out/$tag
for i in 1 2; do
  for v in "$@"; do
    export $var=$v
    timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --no-wire --steps 20 --warmup 5 > gpurun_out/$tag/$v.$i.json 2> gpurun_out/$tag/$v.$i.err || { echo "bench $v failed"; tail -20 gpurun_out/$tag/$v.$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],4), 'ms/step', 'op', round(d['roofline']['kernel_ms'],4))" gpurun_out/$tag/$v.$i.json "$var=$v"
  done
done
