# bucket fold: outputs copied by the scatter, applied-only gather; A/B 8,192-id (1,024 threads) vs 4,096-id (512) buckets
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03x
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py > gpurun_out/r03x/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03x/tests.log; exit 1; }
tail -1 gpurun_out/r03x/tests.log
RP_AMD_LIB=$PWD/abx/librpamd_bk12.so timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py > gpurun_out/r03x/tests12.log 2>&1 || { echo tests12 failed; tail -30 gpurun_out/r03x/tests12.log; exit 1; }
tail -1 gpurun_out/r03x/tests12.log
for rep in 1 2; do
timeout -k 10 300 python3 -u tools/merge_fold_ab.py --label bk13 --only big > gpurun_out/r03x/ab13_$rep.json 2>&1 || { echo ab failed; exit 1; }
RP_AMD_LIB=$PWD/abx/librpamd_bk12.so timeout -k 10 300 python3 -u tools/merge_fold_ab.py --label bk12 --only big > gpurun_out/r03x/ab12_$rep.json 2>&1 || { echo ab12 failed; exit 1; }
done
grep -h '"big"' gpurun_out/r03x/ab1*.json | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['label'], round(d['big']['ms_p50'], 4), round(d['big']['ms_min'], 4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03x/prof13 -o run -- python3 -u tools/merge_fold_ab.py --only big --reps 6 > gpurun_out/r03x/prof13.log 2>&1 || { echo prof failed; exit 1; }
RP_AMD_LIB=$PWD/abx/librpamd_bk12.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03x/prof12 -o run -- python3 -u tools/merge_fold_ab.py --only big --reps 6 > gpurun_out/r03x/prof12.log 2>&1 || { echo prof12 failed; exit 1; }
echo done
