# small host lookups: ring + node tests, api latency leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03t
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_ring_gpu.py tests/test_js_gpu.py tests/test_group_gpu.py > gpurun_out/r03t/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03t/tests.log; exit 1; }
tail -2 gpurun_out/r03t/tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu --no-merge --no-wire --sim-n 0 --sim5-n 0 --batch-log2 20 --steps 2 --warmup 1 > gpurun_out/r03t/b.json 2> gpurun_out/r03t/b.err || { echo bench failed; tail -5 gpurun_out/r03t/b.err; exit 1; }
python3 - gpurun_out/r03t/b.json <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = D["api_latency"]
print("lookup", a["lookup"]["median_us"], "lookupN3", a["lookupN3"]["median_us"], "batch", {k: v["median_us"] for k, v in a["lookupNBatch3"].items()})
PY
