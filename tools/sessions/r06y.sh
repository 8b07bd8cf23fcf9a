# round 6, call y: the bucket fold with the next segment word loaded ahead (librpamd.so) against
# the unrolled rank sort alone (librpamd_mid.so) and neither (librpamd_old.so), 2^22 in place,
# alternating; then the members and partition tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06y}; mkdir -p $O
L=$GRAFT_REPO_ROOT/ringpop-node_amd
for rep in 1 2 3; do
  for lib in librpamd_old.so librpamd_mid.so librpamd.so; do
    RP_AMD_LIB=$L/$lib timeout -k 10 200 python3 -u tools/merge_fold_ab.py --only big --inplace --reps 20 > $O/ab_${lib%.so}_$rep.json 2> $O/ab_${lib%.so}_$rep.err || { echo "ab failed $lib"; tail $O/ab_${lib%.so}_$rep.err; exit 1; }
    echo "$lib rep=$rep $(python3 -c "import json;d=json.load(open('$O/ab_${lib%.so}_$rep.json'))['big'];print(round(d['ms_p50'],5), round(d['ms_min'],5))")"
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_members_gpu.py tests/test_merge_shard_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
