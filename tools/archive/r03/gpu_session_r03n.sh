# C5 refresh kernel A/B: default (lanes / pc32) vs the lane-pair kernel vs k_ck_pc<7,4>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03n
B="python3 -u bench.py --no-cpu --no-api --no-merge --no-wire --sim5-cpu 0 --sim-n 0 --batch-log2 20 --steps 2 --warmup 1"
for v in default pair pc; do
if [ $v = default ]; then E=""; else E="RP_SIM_CK=$v"; fi
env $E timeout -k 10 300 $B > gpurun_out/r03n/c5_$v.json 2> gpurun_out/r03n/c5_$v.err || { echo bench failed; tail -5 gpurun_out/r03n/c5_$v.err; exit 1; }
python3 - gpurun_out/r03n/c5_$v.json $v <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["sim_c5"]; print(sys.argv[2], round(d["ms_per_round"], 2), d["round_ms"])
PY
done
echo done
