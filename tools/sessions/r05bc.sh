# round 5, call bc: the deferred-key pass redoing listed keys from the hashes the lean kernel stored
# (no key reload, no rehash: new) against HEAD, alternating
# in one box; then the ring GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r05bc}; mkdir -p $O
for r in 1 2 3 4; do
  for v in new head; do
    L=; [ $v = head ] && L=$GRAFT_REPO_ROOT/ringpop-node_amd/ab/librpamd_head.so
    RP_AMD_LIB=$L timeout -k 10 240 python3 -u bench.py --no-cpu --no-merge --no-wire --no-api --sim-n 0 --sim5-n 0 > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v rc=$?"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"] / 1e9, 2), "G/s", round(d["ms_per_step"], 4), "ms/step", round(d["roofline"].get("kernel_ms", 0) or 0, 4))
PY
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ring_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
