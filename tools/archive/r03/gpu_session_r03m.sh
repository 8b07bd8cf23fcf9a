# D1 pair kernel: views per group 8 vs 16
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03m
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py -k "d1 or golden" > gpurun_out/r03m/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03m/tests.log; exit 1; }
tail -2 gpurun_out/r03m/tests.log
B="python3 -u bench.py --no-cpu --no-api --no-merge --no-wire --sim5-cpu 0 --sim-n 0 --batch-log2 20 --steps 2 --warmup 1"
for v in 8 16; do
RP_SIM_D1_VPG=$v timeout -k 10 300 $B > gpurun_out/r03m/c5_v$v.json 2> gpurun_out/r03m/c5_v$v.err || { echo bench failed; tail -5 gpurun_out/r03m/c5_v$v.err; exit 1; }
python3 - gpurun_out/r03m/c5_v$v.json $v <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["sim_c5"]; print("vpg", sys.argv[2], round(d["ms_per_round"], 2), d["round_ms"])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03m/prof -o run -- $B > gpurun_out/r03m/c5_prof.json 2> gpurun_out/r03m/c5_prof.err || { echo prof failed; tail -5 gpurun_out/r03m/c5_prof.err; exit 1; }
echo done
