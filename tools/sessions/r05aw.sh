# round 5, call aw: the C2 lookupN(3) bench leg with the lean kernel's ablation branches compiled
# out (new; RP_LOOKUP_HINT=0: new-h0) against HEAD (ab/librpamd_head.so) and the round-4 final
# code (abtree_r04), alternating in one box; then the ring GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r05aw}; mkdir -p $O
for r in 1 2 3; do
  for v in new head r04 newh0; do
    D=$GRAFT_REPO_ROOT; [ $v = r04 ] && D=$GRAFT_REPO_ROOT/abtree_r04
    L=; [ $v = head ] && L=$GRAFT_REPO_ROOT/ringpop-node_amd/ab/librpamd_head.so
    H=; [ $v = newh0 ] && H=0
    (cd $D && RP_AMD_LIB=$L RP_LOOKUP_HINT=$H timeout -k 10 240 python3 -u bench.py --no-cpu --no-merge --no-wire --no-api --sim-n 0 --sim5-n 0) > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v rc=$?"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"] / 1e9, 2), "G/s", round(d["ms_per_step"], 4), "ms/step", round(d["roofline"].get("kernel_ms", 0) or 0, 4))
PY
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ring_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
