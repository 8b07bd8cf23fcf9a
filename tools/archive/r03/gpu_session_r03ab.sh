# checksum string from the names table's address-ordered copy: membership / merge / node tests, C3 merge leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03ab
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py tests/test_js_gpu.py tests/test_damp_gpu.py > gpurun_out/r03ab/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03ab/tests.log; exit 1; }
tail -1 gpurun_out/r03ab/tests.log
timeout -k 10 300 python3 -u tools/merge_fold_ab.py --label r03ab --only c3,c3ck > gpurun_out/r03ab/ab.json 2> gpurun_out/r03ab/ab.err || { echo ab failed; exit 1; }
cat gpurun_out/r03ab/ab.json
for rep in 1 2; do
timeout -k 10 400 python3 -u bench.py --no-cpu --no-api --no-wire --sim-n 0 --sim5-n 0 --steps 2 --warmup 1 > gpurun_out/r03ab/b$rep.json 2> gpurun_out/r03ab/b$rep.err || { echo bench failed; tail -5 gpurun_out/r03ab/b$rep.err; exit 1; }
python3 - gpurun_out/r03ab/b$rep.json <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["merge"]; print("C3", round(d["updates_per_s"]/1e9, 3), "G/s fold", round(d["fold"]["ms_per_batch"], 4), "large", round(d["fold_large"]["ms_per_batch"], 4))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03ab/prof -o run -- python3 -u bench.py --no-cpu --no-api --no-wire --sim-n 0 --sim5-n 0 --steps 2 --warmup 1 > gpurun_out/r03ab/prof.json 2> gpurun_out/r03ab/prof.err || { echo prof failed; exit 1; }
echo done
