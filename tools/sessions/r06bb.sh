# round 6, call bb: the lean kernel's grid, the close candidates alternating over 15 rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06bb}; mkdir -p $O
timeout -k 10 400 python3 -u tools/ab_lookup.py --rounds 15 --only default/lookupN3,grid5120/lookupN3,grid16384/lookupN3,grid32768/lookupN3 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail $O/ab.err; exit 1; }
timeout -k 10 400 python3 -u tools/ab_lookup.py --rounds 15 --only grid32768/lookupN3,grid16384/lookupN3,grid5120/lookupN3,default/lookupN3 > $O/ab2.json 2> $O/ab2.err || { echo "ab2 failed"; tail $O/ab2.err; exit 1; }
python3 tools/show_ab.py $O/ab.json $O/ab2.json
