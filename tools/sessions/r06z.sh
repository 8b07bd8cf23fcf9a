# round 6, call z: the bucket fold with its rows loaded at the start, under the records walk
# (librpamd_rowpf.so, 79 VGPRs + 4 spilled to keep 6 waves a SIMD) against the committed fold
# (librpamd_old.so), 2^22 in place, alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06z}; mkdir -p $O
L=$GRAFT_REPO_ROOT/ringpop-node_amd
for rep in 1 2 3; do
  for lib in librpamd_old.so librpamd_rowpf.so; do
    RP_AMD_LIB=$L/$lib timeout -k 10 200 python3 -u tools/merge_fold_ab.py --only big --inplace --reps 20 > $O/ab_${lib%.so}_$rep.json 2> $O/ab_${lib%.so}_$rep.err || { echo "ab failed $lib"; tail $O/ab_${lib%.so}_$rep.err; exit 1; }
    echo "$lib rep=$rep $(python3 -c "import json;d=json.load(open('$O/ab_${lib%.so}_$rep.json'))['big'];print(round(d['ms_p50'],5), round(d['ms_min'],5))")"
  done
done
