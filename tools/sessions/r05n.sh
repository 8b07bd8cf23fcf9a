# round 5, call n: bucket fold with 8-B records: kernel times (rocprof stats), PMC bytes (copy-out and in place)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 tools/merge_fold_ab.py --only big --reps 9 --inplace > $O/stats.log 2>&1 || { echo "stats failed"; tail -20 $O/stats.log; exit 1; }
find $O/stats -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats_inplace.csv
head -12 $O/kernel_stats_inplace.csv | cut -c1-220
PMC_BK_ARGS=--inplace bash tools/pmc_bk.sh $O/pmc_inplace || exit 1
bash tools/pmc_bk.sh $O/pmc_copy || exit 1
python3 tools/pmc_merge_summary.py $O/pmc_inplace $O/pmc_copy > $O/pmc_summary.json 2>&1
python3 -c "
import json; d=json.load(open('$O/pmc_summary.json'))
for run, ks in d.items():
    tot = 0
    for k, e in ks.items():
        b = e.get('hbm_bytes', 0) / (1 << 22); tot += b if e['grid_threads'] > 10000 else 0
        print(run, k, e['dispatches'], round(b, 2), round(e.get('l2_hit_rate') or 0, 3))
    print(run, 'B/update (large grids)', round(tot, 2))
"
