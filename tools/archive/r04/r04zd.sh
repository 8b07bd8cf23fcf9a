# round 4, call zd: the C2 full-size ring test exact on all 2^24 keys on every layout
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04zd; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread tests/test_ring_gpu.py -k "c2_full_size" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log; grep -c PASSED $O/tests.log
