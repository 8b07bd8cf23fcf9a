# bucket fold: membership tests + merge bench legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03q
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py > gpurun_out/r03q/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03q/tests.log; exit 1; }
tail -2 gpurun_out/r03q/tests.log
B="python3 -u bench.py --no-cpu --no-api --no-wire --sim-n 0 --sim5-n 0 --batch-log2 20 --steps 2 --warmup 1"
for v in 1 0; do
RP_MEMBERS_BUCKET_FOLD=$v timeout -k 10 300 $B > gpurun_out/r03q/m$v.json 2> gpurun_out/r03q/m$v.err || { echo bench failed; tail -5 gpurun_out/r03q/m$v.err; exit 1; }
python3 - gpurun_out/r03q/m$v.json $v <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = D["merge"]; print("bucket", sys.argv[2], "C3", round(d["updates_per_s"]/1e9, 3), "G/s fold", round(d["fold"]["ms_per_batch"], 4), "large", json.dumps(d["fold_large"]))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03q/prof -o run -- $B > gpurun_out/r03q/prof.json 2> gpurun_out/r03q/prof.err || { echo prof failed; tail -5 gpurun_out/r03q/prof.err; exit 1; }
echo done
