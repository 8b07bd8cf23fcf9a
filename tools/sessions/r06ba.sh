# round 6, call ba: the lean kernel's grid re-swept on the final kernel (default 4,096 workgroups)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ba}; mkdir -p $O
timeout -k 10 400 python3 -u tools/ab_lookup.py --rounds 9 --only default/lookupN3,grid1024/lookupN3,grid3072/lookupN3,grid5120/lookupN3,grid6144/lookupN3,grid8192/lookupN3,grid16384/lookupN3 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail $O/ab.err; exit 1; }
python3 tools/show_ab.py $O/ab.json
