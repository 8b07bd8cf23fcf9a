# round 6, call q: the 2^22 bucket fold with 1,024-thread workgroups (-DRP_BK_FT=1024: one tile
# segment a lane, two workgroups and 32 waves a CU) against the 512-thread default, alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06q}; mkdir -p $O
L=$GRAFT_REPO_ROOT/ringpop-node_amd
RP_AMD_LIB=$L/librpamd_ft1024.so timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_members_gpu.py -k "bucket or big or large" > $O/tests_ft1024.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_ft1024.log; exit 1; }
tail -2 $O/tests_ft1024.log
for rep in 1 2 3; do
  for lib in librpamd.so librpamd_ft1024.so; do
    RP_AMD_LIB=$L/$lib timeout -k 10 200 python3 -u tools/merge_fold_ab.py --only big --inplace --reps 20 > $O/ab_${lib%.so}_$rep.json 2> $O/ab_${lib%.so}_$rep.err || { echo "ab failed $lib"; tail $O/ab_${lib%.so}_$rep.err; exit 1; }
    echo "$lib rep=$rep $(cat $O/ab_${lib%.so}_$rep.json)"
  done
done
# the service's device phase stamps with the clock read after the poll's return (one wave)
for a in 1 0; do
  RP_SVC_PROF=1 RP_SVC_WAVES=1 RP_SVC_ANS=$a timeout -k 10 120 node tools/svc_latency.js 10000 4000 8192 > $O/prof_$a.json 2> $O/prof_$a.err || { echo "prof run failed $a"; cat $O/prof_$a.err; exit 1; }
  echo "prof ans=$a $(cat $O/prof_$a.json)"; cat $O/prof_$a.err
done
