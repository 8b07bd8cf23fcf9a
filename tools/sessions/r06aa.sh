# round 6, call aa: C5 round by round with the views hashed per round, with and without the twin
# dedupe (RP_SIM_TWINS=0: every dirty view), for the p95 round's refresh count
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06aa}; mkdir -p $O
timeout -k 10 300 python3 -u tools/c5_rounds.py --label twins > $O/c5_twins.json 2> $O/c5_twins.err || { echo "c5 failed"; tail $O/c5_twins.err; exit 1; }
RP_SIM_TWINS=0 timeout -k 10 300 python3 -u tools/c5_rounds.py --label no-twins > $O/c5_notwins.json 2> $O/c5_notwins.err || { echo "c5 notwins failed"; tail $O/c5_notwins.err; exit 1; }
python3 - $O <<'PY'
import json, sys
a = json.load(open(sys.argv[1] + "/c5_twins.json")); b = json.load(open(sys.argv[1] + "/c5_notwins.json"))
print("rounds", a["rounds"], b["rounds"], "p95", a["p95"], b["p95"], "worst", a["worst"], b["worst"], "chunks/chain", a["chunks_per_chain"])
for x, y in zip(a["per_round"], b["per_round"]):
    print(x["round"], x["ms"], x["views_hashed"], y["ms"], y["views_hashed"])
PY
