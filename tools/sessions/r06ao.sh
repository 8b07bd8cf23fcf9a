# round 6, call ao: after the PartMembership.partition refactor: the merge-shard and bench tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ao}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_merge_shard_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
