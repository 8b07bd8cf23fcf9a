# round 5, call t: the whole GPU suite and smoke() on the code as it stands (O overridable)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05t}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
