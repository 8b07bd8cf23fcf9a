# round 6, call d: the LDS-index kernel's time ablations and staging A/B against the lean kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06d}; mkdir -p $O
timeout -k 10 300 python3 -u tools/ab_lookup.py --rounds 5 --only lean/lookupN3,lds/lookupN3,lds-stg1/lookupN3,lds-abl1/lookupN3,lds-abl2/lookupN3,lds-abl3/lookupN3,lds-abl4/lookupN3,lds-abl7/lookupN3 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json'))
for k,v in d.items(): print('%-22s %.4f ms  %.1f G/s' % (k, v['median_ms'], v['Glookups_s']))
"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "lds" > $O/ring_lds.log 2>&1 || { echo "ring lds failed"; tail -30 $O/ring_lds.log; exit 1; }
tail -1 $O/ring_lds.log
# the sharded simulator's exchange per round, round 5 tree (host barriers in rp_sim_outbox /
# rp_sim_inbox) against this one, 4 gloo ranks on the box's GPU, alternating
for r in 1 2; do
  for v in r05 new; do
    B=bench.py; [ $v = r05 ] && B=abtree_r05/bench.py
    RP_BENCH_BACKEND=gloo timeout -k 10 240 python3 -u $B --gpus 4 --steps 2 --warmup 1 --batch-log2 18 --no-merge --no-wire --no-cpu --no-api --sim-n 0 --sim5-n 3000 > $O/x_${v}_$r.json 2> $O/x_${v}_$r.err || { echo "$v rc=$?"; tail -5 $O/x_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/x_${v}_$r.json').read().strip().splitlines()[-1])['sim_c5']
print('$v', {k: (round(v,4) if isinstance(v,float) else v) for k,v in d.items() if k.startswith('exchange') or k in ('rounds',)}, 'round_ms', d['round_ms'])
"
  done
done
