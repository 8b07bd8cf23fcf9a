# sim changes: due-prefix timers, DPP pair block_checksum, change-list hash in block_apply
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03j
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py tests/test_sim_digests_gpu.py tests/test_sim_shard_gpu.py > gpurun_out/r03j/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03j/tests.log; exit 1; }
tail -2 gpurun_out/r03j/tests.log
B="python3 -u bench.py --no-cpu --no-api --no-merge --no-wire --sim5-cpu 0 --batch-log2 20 --steps 2 --warmup 1"
timeout -k 10 300 $B > gpurun_out/r03j/c5_default.json 2> gpurun_out/r03j/c5_default.err || { echo bench failed; tail -5 gpurun_out/r03j/c5_default.err; exit 1; }

for f in c5_default; do python3 - gpurun_out/r03j/$f.json $f <<'PY'
import json, sys
D = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("sim", "sim_c5"):
    d = D[k]; print(sys.argv[2], k, round(d["ms_per_round"], 2), d["round_ms"], d["rounds_to_convergence"])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03j/prof -o run -- $B > gpurun_out/r03j/c5_prof.json 2> gpurun_out/r03j/c5_prof.err || { echo prof failed; tail -5 gpurun_out/r03j/c5_prof.err; exit 1; }
echo done
