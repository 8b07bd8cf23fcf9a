# 4,096-id bucket fold default: full GPU suite, fold A/B, merge leg of the bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03y
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r03y/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03y/tests.log; exit 1; }
tail -1 gpurun_out/r03y/tests.log
timeout -k 10 300 python3 -u tools/merge_fold_ab.py --label r03y > gpurun_out/r03y/ab.json 2> gpurun_out/r03y/ab.err || { echo ab failed; exit 1; }
cat gpurun_out/r03y/ab.json
timeout -k 10 400 python3 -u bench.py --no-cpu --no-api --no-wire --sim-n 0 --sim5-n 0 --steps 2 --warmup 1 > gpurun_out/r03y/b.json 2> gpurun_out/r03y/b.err || { echo bench failed; tail -5 gpurun_out/r03y/b.err; exit 1; }
python3 - gpurun_out/r03y/b.json <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["merge"]; print("C3", round(d["updates_per_s"]/1e9, 3), "G/s fold", round(d["fold"]["ms_per_batch"], 4), "large", round(d["fold_large"]["ms_per_batch"], 4), round(d["fold_large"]["roofline"]["frac"], 4))
PY
echo done
