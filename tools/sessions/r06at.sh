# round 6, call at: the wave-specialised lookupN kernel (k_lookupn_ws, RP_LOOKUP_WS): parity on every
# ring test with ws layouts, then an alternating A/B against the lean kernel in one process
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06at}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ring_gpu.py -k "ws" > $O/tests_ws.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_ws.log; exit 1; }
tail -1 $O/tests_ws.log
RP_LOOKUP_DEBUG=1 timeout -k 10 120 python3 -u tools/ab_lookup.py --rounds 1 --only ws13/lookupN3,ws412/lookupN3 > $O/ab_debug.json 2> $O/ab_debug.err || { echo "debug failed"; tail $O/ab_debug.err; exit 1; }
grep "ws lookupN" $O/ab_debug.err | head -4
timeout -k 10 400 python3 -u tools/ab_lookup.py --rounds 9 --only default/lookupN3,ws13/lookupN3,ws26/lookupN3,ws17/lookupN3,ws412/lookupN3,ws13-g512/lookupN3,ws13-g2048/lookupN3 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail $O/ab.err; exit 1; }
python3 tools/show_ab.py $O/ab.json
