# round 6, call aq: the D1 sender chains grouped by string-length delta (RP_SIM_D1_SORT=1) against
# list order, C5 per round alternating; digests with it on
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06aq}; mkdir -p $O
for rep in 1 2; do
  for v in 0 1; do
    RP_SIM_D1_SORT=$v timeout -k 10 300 python3 -u tools/c5_rounds.py --label d1s$v > $O/c5_d1s${v}_$rep.json 2> $O/c5_d1s${v}_$rep.err || { echo "c5 failed $v"; tail $O/c5_d1s${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5_d1s${v}_$rep.json'));ms=[x['ms'] for x in d['per_round']];print('d1sort=$v rep=$rep rounds',d['rounds'],'mean %.2f p50 %.1f p95 %.2f max %.1f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
  done
done
RP_SIM_D1_SORT=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sim_digests_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
