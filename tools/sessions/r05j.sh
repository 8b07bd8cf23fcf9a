# round 5, call j: windows as an aligned dwordx4 + dword (RP_LOOKUP_AL): parity on the lookup
# layouts, then A/B against the kept kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ring_gpu.py -k "al or compact" > $O/ring.log 2>&1 || { echo "ring tests failed"; tail -40 $O/ring.log; exit 1; }
tail -2 $O/ring.log
timeout -k 10 400 python -u tools/ab_lk.py --rounds 11 --out $O/ab.json --variants '{"base": {}, "al": {"RP_LOOKUP_AL": "1"}, "al-a1": {"RP_LOOKUP_AL": "1", "RP_LOOKUP_ABLATE": "1"}, "a1": {"RP_LOOKUP_ABLATE": "1"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -30 $O/ab.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json'))
for k,v in d.items(): print(k, v['median_ms'], v['min_ms'], v['hbm_frac'], v['same_as_base'])"
