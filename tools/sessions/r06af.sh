# round 6, call af: the simulator suites with the sorted refresh order as the default (C4/C5
# digests, sharded, goldens) and the C5 bench leg alone
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06af}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_sim_digests_gpu.py tests/test_sim_gpu.py tests/test_sim_shard_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/c5_rounds.py --label default > $O/c5_default.json 2> $O/c5_default.err || { echo "c5 failed"; tail $O/c5_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5_default.json'));ms=[x['ms'] for x in d['per_round']];print('default rounds',d['rounds'],'mean %.1f p50 %.1f p95 %.1f max %.1f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
