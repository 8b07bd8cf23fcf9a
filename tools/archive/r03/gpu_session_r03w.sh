# bucket fold without the count pass: tile-contiguous record runs, LDS payload fold, resid gather
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03w
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py > gpurun_out/r03w/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03w/tests.log; exit 1; }
tail -2 gpurun_out/r03w/tests.log
timeout -k 10 300 python3 -u tools/merge_fold_ab.py --label r03w --only big,c3 > gpurun_out/r03w/ab.json 2> gpurun_out/r03w/ab.err || { echo ab failed; tail -5 gpurun_out/r03w/ab.err; exit 1; }
cat gpurun_out/r03w/ab.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03w/prof -o run -- python3 -u tools/merge_fold_ab.py --label r03w --only big --reps 6 > gpurun_out/r03w/prof.json 2> gpurun_out/r03w/prof.err || { echo prof failed; tail -5 gpurun_out/r03w/prof.err; exit 1; }
f=$(find gpurun_out/r03w/prof -name '*kernel_stats.csv' | head -1); grep -E "k_bk|k_fold_ovf|Name" $f | cut -c1-40,100-220
echo done
