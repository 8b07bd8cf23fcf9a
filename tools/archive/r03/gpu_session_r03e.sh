mkdir -p gpurun_out/mab
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ > gpurun_out/mab/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/mab/tests.log; exit 1; }
tail -2 gpurun_out/mab/tests.log
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 240 python3 -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --batch-log2 20 --steps 2 --warmup 1 > gpurun_out/mab/$tag.json 2> gpurun_out/mab/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/mab/$tag.err; return 1; }
  python3 - gpurun_out/mab/$tag.json $tag <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["merge"]
print(sys.argv[2], round(d["updates_per_s"] / 1e6, 1), "M/s", round(d["ms_per_batch"], 4), "ms/batch", "fold", round(d["fold"]["ms_per_batch"], 4), "chain", round(d["checksum_chain"]["ms"], 3))
print("wire", json.dumps(D.get("wire"))[:600])
PY
}
run base RP_X=1
bash tools/gpu_session_r03f.sh | tail -32
