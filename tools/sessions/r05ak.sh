# round 5, call ak: k_bk_fold phase cycle counters with 8-B rows and records (ab/librpamd_bkprof.so, -DRP_BK_PROF) over 2^22 batches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ak; mkdir -p $O
RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_bkprof.so RP_BK_PROF_PRINT=1 timeout -k 10 200 python -u tools/ab_fold.py --rounds 6 --out $O/prof.json --variants '{"direct": {"INPLACE": "1"}}' > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
grep "k_bk_fold cycles" $O/prof.log | tail -5
python3 -c "import json;d=json.load(open('$O/prof.json'))['direct'];print(d)"
