# round 6, call v: the id-partitioned 2^22 fold's per-rank work (tools/part_fold.py: 1/G of the
# buckets for G = 1, 2, 4, 8, alternating) and bench.py --gpus 4 (gloo, ranks sharing the GPU)
# with the partitioned leg (tests/test_bench_gpu.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06v}; mkdir -p $O
timeout -k 10 300 python3 -u tools/part_fold.py --reps 12 > $O/part_fold.json 2> $O/part_fold.err || { echo "part_fold failed"; tail -20 $O/part_fold.err; exit 1; }
cat $O/part_fold.json
timeout -k 10 600 python3 -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu tests/test_bench_gpu.py > $O/tests_bench.log 2>&1 || { echo "bench tests failed"; tail -40 $O/tests_bench.log; exit 1; }
grep -E "passed|failed" $O/tests_bench.log | tail -2
