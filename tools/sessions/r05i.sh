# round 5, call i: what the window's cost is made of: dword-aligned windows (RP_LOOKUP_ABLATE=16,
# results wrong) against 16-B-aligned (2) and the kept kernel, alternating in one process
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 400 python -u tools/ab_lk.py --rounds 9 --out $O/ab.json --variants '{"base": {}, "a16": {"RP_LOOKUP_ABLATE": "16"}, "a2": {"RP_LOOKUP_ABLATE": "2"}, "a1": {"RP_LOOKUP_ABLATE": "1"}, "a17": {"RP_LOOKUP_ABLATE": "17"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -30 $O/ab.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json'))
for k,v in d.items(): print(k, v['median_ms'], v['min_ms'], v['hbm_frac'])"
