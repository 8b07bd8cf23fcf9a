# round 5, call ai: compact bucket density (RP_COMPACT_CB_DELTA -1: half the buckets, a 256-KB hinted
# index, ~3.8 tokens per bucket) against the kept cb = floor(log2 M), lookupN(3) at 2^26, alternating processes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ai; mkdir -p $O
for r in 1 2 3; do
  for v in base m1; do
    if [ $v = m1 ]; then export RP_COMPACT_CB_DELTA=-1; else unset RP_COMPACT_CB_DELTA; fi
    timeout -k 10 200 python -u tools/ab_lk.py --rounds 7 --out $O/${v}_$r.json --variants '{"lk": {}}' > $O/${v}_$r.log 2>&1 || { echo "ab $v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'))['lk'];print('$v $r', d['median_ms'], d['min_ms'], d['hbm_frac'])"
  done
done
