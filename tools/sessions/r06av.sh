# round 6, call av: the wave-specialised lookupN kernel with more consumer waves a CU (1:15, 2:14
# in one 16-wave workgroup) against 4:12 and the lean kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06av}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ring_gpu.py -k "ws" > $O/tests_ws.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_ws.log; exit 1; }
tail -1 $O/tests_ws.log
timeout -k 10 400 python3 -u tools/ab_lookup.py --rounds 9 --only default/lookupN3,ws412/lookupN3,ws115/lookupN3,ws214/lookupN3 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail $O/ab.err; exit 1; }
python3 tools/show_ab.py $O/ab.json
