# round 5, call at: the C3 merge leg with the checksum chains' stream confined to n CUs
# (RP_MEMBERS_CK_CUS; 0 = all), alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05at}; mkdir -p $O
for r in 1 2; do
  for v in 0 64 128 192; do
    RP_MEMBERS_CK_CUS=$v timeout -k 10 240 python3 -u bench.py --no-cpu --no-wire --no-api --sim-n 0 --sim5-n 0 \
        --batch-log2 20 --steps 2 --warmup 1 > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v rc=$?"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["merge"]
print(sys.argv[2], round(d["updates_per_s"] / 1e6, 1), "M/s", round(d["ms_per_batch"], 4), "ms/batch", d["checksum"])
PY
  done
done
