# round 5, call c: the 2^22 bucket fold with early row loads + two segments a lane (RP_BK_PRE) and
# the 16-wide gather (RP_BK_GV): members tests on every fold path, A/B in one process
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_members_gpu.py > $O/members.log 2>&1 || { echo "members tests failed"; tail -40 $O/members.log; exit 1; }
tail -2 $O/members.log
timeout -k 10 300 python -u tools/ab_fold.py --rounds 8 --out $O/ab.json --variants '{"new": {}, "old": {"RP_BK_PRE": "0", "RP_BK_GV": "4"}, "pre-gv4": {"RP_BK_GV": "4"}, "pre0-gv16": {"RP_BK_PRE": "0"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -30 $O/ab.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json'))
for k,v in d.items(): print(k, v['median_ms'], v['min_ms'], v['frac_49B'])"
