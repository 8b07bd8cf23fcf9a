# round 5, call ab: PMC HBM bytes of the 2^22 bucket fold with 8-B member rows (in place and copy-out)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab; mkdir -p $O
PMC_BK_ARGS=--inplace bash tools/pmc_bk.sh $O/pmc_inplace || exit 1
bash tools/pmc_bk.sh $O/pmc_copy || exit 1
python3 tools/pmc_merge_summary.py $O/pmc_inplace $O/pmc_copy > $O/pmc_summary.json 2>&1
python3 -c "
import json; d=json.load(open('$O/pmc_summary.json'))
for run, ks in d.items():
    tot = 0
    for k, e in ks.items():
        if 'bk_' in k or 'fold_ovf' in k:
            b = e.get('hbm_bytes', 0) / (1 << 22); tot += b
            print(run, k, e['dispatches'], round(b, 2), round(e.get('l2_hit_rate') or 0, 3))
    print(run, 'bucket path B/update', round(tot, 2))
"
rm -rf $O/pmc_inplace/*/ $O/pmc_copy/*/
