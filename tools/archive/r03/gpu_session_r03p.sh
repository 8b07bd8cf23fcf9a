# k_pass1 ahead of the refresh kernels: sim tests + C5 A/B (RP_SIM_PASS1=0 / default)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03p
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py tests/test_sim_digests_gpu.py > gpurun_out/r03p/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03p/tests.log; exit 1; }
tail -2 gpurun_out/r03p/tests.log
B="python3 -u bench.py --no-cpu --no-api --no-merge --no-wire --sim5-cpu 0 --batch-log2 20 --steps 2 --warmup 1"
for v in 1 0; do
RP_SIM_PASS1=$v timeout -k 10 300 $B > gpurun_out/r03p/c5_p$v.json 2> gpurun_out/r03p/c5_p$v.err || { echo bench failed; tail -5 gpurun_out/r03p/c5_p$v.err; exit 1; }
python3 - gpurun_out/r03p/c5_p$v.json $v <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("sim", "sim_c5"):
    d = D[k]; print("pass1", sys.argv[2], k, round(d["ms_per_round"], 2), d["round_ms"])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03p/prof -o run -- $B > gpurun_out/r03p/c5_prof.json 2> gpurun_out/r03p/c5_prof.err || { echo prof failed; tail -5 gpurun_out/r03p/c5_prof.err; exit 1; }
echo done
