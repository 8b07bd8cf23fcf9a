# round 5, call av: the C2 lookupN(3) bench leg of HEAD against the round-4 final code
# (abtree_r04: git archive c8ba035, built here), alternating in one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r05av}; mkdir -p $O
for r in 1 2 3; do
  for v in head r04; do
    D=$GRAFT_REPO_ROOT; [ $v = r04 ] && D=$GRAFT_REPO_ROOT/abtree_r04
    (cd $D && timeout -k 10 240 python3 -u bench.py --no-cpu --no-merge --no-wire --no-api --sim-n 0 --sim5-n 0) > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v rc=$?"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"] / 1e9, 2), "G/s", round(d["ms_per_step"], 4), "ms/step", round(d["roofline"].get("kernel_ms", 0) or 0, 4))
PY
  done
done
