# round 4, call i: wire decoder records parsed a lane per member (-DRP_WIRE_MEMBERS=1, in-tree)
# against the per-record lane walk (ab/librpamd_base.so, -DRP_WIRE_MEMBERS=0): wire + JS GPU
# tests on the new build, then the wire leg alternating the two libraries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i; mkdir -p $O
: timeout -k 10 300 python -u -m pytest tests/test_js_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/jstest.log 2>&1 || { echo js tests failed; tail -30 $O/jstest.log; exit 1; }
: tail -1 $O/jstest.log
bash tools/ab_wire.sh r04i
