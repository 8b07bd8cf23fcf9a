# round 6, call ae: C5 refresh order A/B, alternating: default (0), ordered by this round's shifts
# after a pass-1 launch (1), by the string-length delta kept per view (3); then the C4/C5 digest
# tests with mode 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ae}; mkdir -p $O
for rep in 1 2; do
  for v in 0 1 3; do
    RP_SIM_CK_SORT=$v timeout -k 10 300 python3 -u tools/c5_rounds.py --label sort$v > $O/c5_sort${v}_$rep.json 2> $O/c5_sort${v}_$rep.err || { echo "c5 failed $v"; tail $O/c5_sort${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5_sort${v}_$rep.json'));ms=[x['ms'] for x in d['per_round']];print('sort=$v rep=$rep rounds',d['rounds'],'mean %.1f p50 %.1f p95 %.1f max %.1f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
  done
done
RP_SIM_CK_SORT=3 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sim_digests_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
