# round 6, call j: the deferred string write (batch b's string in batch b + 1's fold launch):
# membership parity, then the C3 stream A/B against the build-stream and inline forms
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06j}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py tests/test_damp_gpu.py > $O/members.log 2>&1 || { echo "members failed"; tail -40 $O/members.log; exit 1; }
tail -1 $O/members.log
timeout -k 10 700 python3 -u tools/c3_ab.py --batches 1024 --rounds 3 --variants fused,side,noside,fused-g512 > $O/c3ab.log 2>&1 || { echo "c3ab failed"; tail -20 $O/c3ab.log; exit 1; }
grep -v "^{" $O/c3ab.log
