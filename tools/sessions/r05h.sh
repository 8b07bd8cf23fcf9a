# round 5, call h: line-aligned compact entries for the lean lookupN(3) (k_pack18, RP_LOOKUP_L18):
# every lookup layout + the exact C2 test, then A/B (with / without L18 and hints)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ring_gpu.py > $O/ring.log 2>&1 || { echo "ring tests failed"; tail -40 $O/ring.log; exit 1; }
tail -2 $O/ring.log
timeout -k 10 400 python -u tools/ab_lk.py --rounds 9 --out $O/ab.json --variants '{"l18": {}, "l18off": {"RP_LOOKUP_L18": "0"}, "l18-hint0": {"RP_LOOKUP_HINT": "0"}, "l18off-hint0": {"RP_LOOKUP_L18": "0", "RP_LOOKUP_HINT": "0"}, "l18-a1": {"RP_LOOKUP_ABLATE": "1"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -30 $O/ab.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json'))
for k,v in d.items(): print(k, v['median_ms'], v['min_ms'], v['hbm_frac'], v['same_as_l18'])"
