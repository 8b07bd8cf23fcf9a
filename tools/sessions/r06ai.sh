# round 6, call ai: C5 split into 8 shards inside one process on the one GPU (ShardedGossipSim;
# each shard refreshes on the producer/consumer path, as each rank of an 8-GPU run does), with
# and without the sorted order there (RP_SIM_CK_SORT_PC), alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ai}; mkdir -p $O
for rep in 1 2; do
  for v in 0 1; do
    RP_SIM_CK_SORT_PC=$v timeout -k 10 400 python3 -u tools/c5_rounds.py --shards 8 --label sh8pc$v > $O/c5s8_pc${v}_$rep.json 2> $O/c5s8_pc${v}_$rep.err || { echo "c5 sharded failed $v"; tail $O/c5s8_pc${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5s8_pc${v}_$rep.json'));ms=[x['ms'] for x in d['per_round']];print('pc_sort=$v rep=$rep rounds',d['rounds'],'mean %.1f p50 %.1f p95 %.1f max %.1f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
  done
done
