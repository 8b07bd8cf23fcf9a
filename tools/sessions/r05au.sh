# round 5, call au: the C3 merge leg with the checksum strings stored non-temporally and read
# non-temporally by the chains (new) against HEAD, alternating; then the members GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05au}; mkdir -p $O
for r in 1 2 3; do
  for v in new head; do
    L=$PWD/ringpop-node_amd/librpamd.so; [ $v != new ] && L=$PWD/ringpop-node_amd/ab/librpamd_$v.so
    RP_AMD_LIB=$L timeout -k 10 240 python3 -u bench.py --no-cpu --no-wire --no-api --sim-n 0 --sim5-n 0 \
        --batch-log2 20 --steps 2 --warmup 1 > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v rc=$?"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["merge"]
print(sys.argv[2], round(d["updates_per_s"] / 1e6, 1), "M/s", round(d["ms_per_batch"], 4), "ms/batch", round(d["fold"]["ms_per_batch"], 4), d["checksum"])
PY
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_members_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
