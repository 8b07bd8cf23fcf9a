# round 5, call a: tail prefetch of the next tile's keys (RP_LOOKUP_PF) parity + A/B, lean-kernel
# ablations (RP_LOOKUP_ABLATE bits: 1 no second windows, 2 windows inside one line, 4 no index trip,
# 8 no window trip) to price each trip in the current kernel; wire decoder tests against the
# contract oracle
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wire_gpu.py > $O/wire.log 2>&1; echo "wire rc $?"; tail -3 $O/wire.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sim_shard_gpu.py > $O/shard.log 2>&1; echo "shard rc $?"; tail -3 $O/shard.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ring_gpu.py -k "pf" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/ab_lk.py --rounds 7 --out $O/ab.json --variants '{"base": {}, "pf": {"RP_LOOKUP_PF": "1"}, "a1": {"RP_LOOKUP_ABLATE": "1"}, "a2": {"RP_LOOKUP_ABLATE": "2"}, "a4": {"RP_LOOKUP_ABLATE": "4"}, "a8": {"RP_LOOKUP_ABLATE": "8"}, "a12": {"RP_LOOKUP_ABLATE": "12"}, "a3fix": {"RP_LOOKUP_ABLATE": "3"}, "pf-a1": {"RP_LOOKUP_PF": "1", "RP_LOOKUP_ABLATE": "1"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -30 $O/ab.log; exit 1; }
tail -80 $O/ab.log
