# prefetching bucket kernels + pre-sized sim message buffers: tests, merge + sim legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03s
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_sim_gpu.py tests/test_sim_digests_gpu.py > gpurun_out/r03s/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03s/tests.log; exit 1; }
tail -2 gpurun_out/r03s/tests.log
B="python3 -u bench.py --no-cpu --no-api --no-wire --sim5-cpu 0 --batch-log2 20 --steps 2 --warmup 1"
timeout -k 10 400 $B > gpurun_out/r03s/b.json 2> gpurun_out/r03s/b.err || { echo bench failed; tail -5 gpurun_out/r03s/b.err; exit 1; }
python3 - gpurun_out/r03s/b.json <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["merge"]; print("C3", round(d["updates_per_s"]/1e9, 3), "G/s fold", round(d["fold"]["ms_per_batch"], 4), "large", round(d["fold_large"]["ms_per_batch"], 4), round(d["fold_large"]["roofline"]["frac"], 4))
for k in ("sim", "sim_c5"):
    d = D[k]; print(k, round(d["ms_per_round"], 2), d["round_ms"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03s/prof -o run -- python3 -u bench.py --no-cpu --no-api --no-wire --sim-n 0 --sim5-n 0 --batch-log2 20 --steps 2 --warmup 1 > gpurun_out/r03s/prof.json 2> gpurun_out/r03s/prof.err || { echo prof failed; tail -5 gpurun_out/r03s/prof.err; exit 1; }
echo done
