# round 5, call b: the hinted index (per-bucket window-start hints, lookupN(3)): parity on every
# lookup layout + the C2 full-size test, A/B against RP_LOOKUP_HINT=0; the service + batch test
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ring_gpu.py > $O/ring.log 2>&1 || { echo "ring tests failed"; tail -40 $O/ring.log; exit 1; }
tail -3 $O/ring.log
timeout -k 10 300 python -u tools/ab_lk.py --rounds 9 --out $O/ab.json --variants '{"hint": {}, "hint0": {"RP_LOOKUP_HINT": "0"}, "hint-a1": {"RP_LOOKUP_ABLATE": "1"}, "hint0-a1": {"RP_LOOKUP_HINT": "0", "RP_LOOKUP_ABLATE": "1"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -30 $O/ab.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json'))
for k,v in d.items(): print(k, v['median_ms'], v['min_ms'], v['hbm_frac'], v['same_as_hint'])"
