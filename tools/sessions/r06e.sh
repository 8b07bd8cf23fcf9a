# round 6, call e: the C3 string writer on a build stream from a rank-ordered row snapshot
# (RP_MEMBERS_SIDE_BUILD, default on) — membership parity, then the C3 stream A/B with chain
# groups of 128 / 256
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06e}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py tests/test_damp_gpu.py > $O/members.log 2>&1 || { echo "members failed"; tail -40 $O/members.log; exit 1; }
tail -1 $O/members.log
timeout -k 10 500 python3 -u tools/c3_ab.py --batches 1024 --rounds 2 --variants noside,side,noside-g256,side-g256 > $O/c3ab.log 2>&1 || { echo "c3ab failed"; tail -20 $O/c3ab.log; exit 1; }
grep -v "^{" $O/c3ab.log
