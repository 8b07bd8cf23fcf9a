# round 4, call d: bucket size A/B for the 2^22 fold (4,096-id buckets, 512-thread folds = main;
# 2,048-id buckets with 512 or 256 threads)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d; mkdir -p $O
for i in 1 2 3; do
  for lib in ringpop-node_amd/librpamd.so ringpop-node_amd/ab/librpamd_bits11.so ringpop-node_amd/ab/librpamd_bits11ft256.so; do
    RP_AMD_LIB=$lib timeout -k 10 200 python3 -u tools/merge_fold_ab.py --only big --reps 20 >> $O/fold_ab.jsonl 2>> $O/fold_ab.err || { echo fold ab failed; tail -20 $O/fold_ab.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/fold_ab.jsonl'):
    d=json.loads(l); print(d['label'].split('/')[-1], round(d['big']['ms_mean'],4), round(d['big']['ms_p50'],4), d['big']['applied_last'])"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c3 -o run -- python3 -u tools/c3_timeline.py run 300 > $O/c3_run.log 2>&1 || { echo c3 run failed; tail -20 $O/c3_run.log; exit 1; }
tail -2 $O/c3_run.log
python3 tools/c3_timeline.py show $O/c3/run_results.db > $O/c3_show.txt 2>&1; tail -45 $O/c3_show.txt
