# round 6, call c: the LDS-index lookup kernel (full-group fix) parity and A/B; sharded sim tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06c}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ring_gpu.py -k "lds or lean" > $O/ring_lds.log 2>&1 || { echo "ring lds failed"; tail -40 $O/ring_lds.log; exit 1; }
tail -1 $O/ring_lds.log
RP_LOOKUP_DEBUG=1 timeout -k 10 200 python3 -u tools/ab_lookup.py --rounds 7 --only lds/lookupN3,lean/lookupN3,lds/lookup,lean/lookup,lds-g512/lookupN3 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
cat $O/ab.json; tail -4 $O/ab.err
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sim_shard_gpu.py tests/test_merge_shard_gpu.py tests/test_bench_gpu.py > $O/shard.log 2>&1 || { echo "shard failed"; tail -40 $O/shard.log; exit 1; }
tail -1 $O/shard.log
