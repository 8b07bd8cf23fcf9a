# k_ck_lanes: production + chain in one basic block (ballot-uniform full groups); sim tests, first 12 C5 rounds traced, C5 leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03z
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py tests/test_sim_digests_gpu.py > gpurun_out/r03z/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03z/tests.log; exit 1; }
tail -1 gpurun_out/r03z/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r03z/p0 -o run -- python3 -u tools/sim_c5_probe.py 100000 12 > gpurun_out/r03z/p0.log 2>&1 || { echo prof failed; tail -5 gpurun_out/r03z/p0.log; exit 1; }
timeout -k 10 500 python3 -u bench.py --no-cpu --no-api --no-wire --no-merge --sim-n 0 --sim5-cpu 0 --steps 2 --warmup 1 > gpurun_out/r03z/b.json 2> gpurun_out/r03z/b.err || { echo bench failed; tail -5 gpurun_out/r03z/b.err; exit 1; }
python3 - gpurun_out/r03z/b.json <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["sim_c5"]; print("c5", round(d["ms_per_round"], 2), d["round_ms"], d.get("rounds"))
PY
echo done
