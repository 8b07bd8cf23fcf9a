# round 5, call y: the scatter with the next tile's inputs loaded under the current tile's stores
# (RP_BK_SGRID workgroups looping over tiles): members GPU tests at 512, then fold A/B (in place)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y; mkdir -p $O
RP_BK_SGRID=512 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_members_gpu.py -k "bucket" > $O/tests512.log 2>&1 || { echo "tests failed"; tail -30 $O/tests512.log; exit 1; }
RP_BK_SGRID=100 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_members_gpu.py -k "bucket" > $O/tests100.log 2>&1 || { echo "tests100 failed"; tail -30 $O/tests100.log; exit 1; }
tail -1 $O/tests512.log; tail -1 $O/tests100.log
timeout -k 10 300 python -u tools/ab_fold.py --rounds 10 --out $O/ab.json --variants '{"one": {"INPLACE": "1"}, "g512": {"INPLACE": "1", "RP_BK_SGRID": "512"}, "g384": {"INPLACE": "1", "RP_BK_SGRID": "384"}, "g256": {"INPLACE": "1", "RP_BK_SGRID": "256"}}' > $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/ab.json'));print({k:(v['median_ms'],v['min_ms']) for k,v in d.items()})"
