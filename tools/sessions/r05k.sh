# round 5, call k: bucket fold with 8,192-change scatter tiles (ab/librpamd_t8k.so, -DRP_BK_TILE=8192:
# half the segments, ~8 records each) against the in-tree 4,096: members tests on the variant, then
# fold legs alternating between the two libraries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05k; mkdir -p $O
A=$PWD/ringpop-node_amd/ab
RP_AMD_LIB=$A/librpamd_t8k.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_members_gpu.py > $O/members_t8k.log 2>&1 || { echo "members tests (t8k) failed"; tail -40 $O/members_t8k.log; exit 1; }
tail -2 $O/members_t8k.log
for i in 1 2 3; do
  for v in tree t8k; do
    if [ $v = tree ]; then unset RP_AMD_LIB; else export RP_AMD_LIB=$A/librpamd_$v.so; fi
    timeout -k 10 200 python -u tools/ab_fold.py --rounds 6 --out $O/$v$i.json --variants '{"direct": {}}' > $O/$v$i.log 2>&1 || { echo "fold $v failed"; tail -20 $O/$v$i.log; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]))['direct'];print(sys.argv[2], d['median_ms'], d['min_ms'], d['frac_49B'])" $O/$v$i.json $v
  done
done
