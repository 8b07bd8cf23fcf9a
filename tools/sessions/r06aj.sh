# round 6, call aj: the simulator suites with the sorted order on sharded handles by default; C5
# in 8 shards on one GPU and C4 per round with the defaults
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06aj}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sim_digests_gpu.py tests/test_sim_shard_gpu.py tests/test_sim_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 -u tools/c5_rounds.py --shards 8 --label sh8 > $O/c5s8.json 2> $O/c5s8.err || { echo "c5 sharded failed"; tail $O/c5s8.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5s8.json'));ms=[x['ms'] for x in d['per_round']];print('c5 8 shards rounds',d['rounds'],'mean %.1f p50 %.1f p95 %.1f max %.1f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
timeout -k 10 300 python3 -u tools/c5_rounds.py --n 10000 --label c4 > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; tail $O/c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c4.json'));ms=[x['ms'] for x in d['per_round']];print('c4 rounds',d['rounds'],'mean %.2f p50 %.2f p95 %.2f max %.2f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
