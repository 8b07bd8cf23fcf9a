# round 6, call h: the packed chain kernel (k_hash_long_pack, 16 strings a workgroup): parity
# (multi-string test, C3 and checksum-group tests), then the C3 stream A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06h}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "long_hash_multi" > $O/hl.log 2>&1 || { echo "hl failed"; tail -30 $O/hl.log; exit 1; }
tail -1 $O/hl.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_members_gpu.py tests/test_merge_shard_gpu.py > $O/members.log 2>&1 || { echo "members failed"; tail -30 $O/members.log; exit 1; }
tail -1 $O/members.log
timeout -k 10 600 python3 -u tools/c3_ab.py --batches 1024 --rounds 2 --variants nopack,side,g256,g512 > $O/c3ab.log 2>&1 || { echo "c3ab failed"; tail -20 $O/c3ab.log; exit 1; }
grep -v "^{" $O/c3ab.log
