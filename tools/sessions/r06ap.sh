# round 6, call ap: a range update past the table (a rank with no ids) folds nothing: the
# partitioned-merge tests incl. 3 ranks over a 2-bucket table, and the members suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ap}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_merge_shard_gpu.py tests/test_members_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
grep -E "part_membership|passed|failed" $O/tests.log | tail -5
