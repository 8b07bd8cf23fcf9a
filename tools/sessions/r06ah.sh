# round 6, call ah: the sorted refresh order on the producer/consumer path (RP_SIM_CK_SORT_PC=1)
# against its default walk: C4 (10k views, one GPU) per round, alternating; digests with it on
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ah}; mkdir -p $O
for rep in 1 2 3; do
  for v in 0 1; do
    RP_SIM_CK_SORT_PC=$v timeout -k 10 300 python3 -u tools/c5_rounds.py --n 10000 --label pc$v > $O/c4_pc${v}_$rep.json 2> $O/c4_pc${v}_$rep.err || { echo "c4 failed $v"; tail $O/c4_pc${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c4_pc${v}_$rep.json'));ms=[x['ms'] for x in d['per_round']];print('pc_sort=$v rep=$rep rounds',d['rounds'],'mean %.2f p50 %.2f p95 %.2f max %.2f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
  done
done
RP_SIM_CK_SORT_PC=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sim_digests_gpu.py tests/test_sim_shard_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
