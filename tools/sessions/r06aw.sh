# round 6, call aw: where the wave-specialised kernel's time goes: 4:12 with producers that load no
# keys (abl1) and with consumers that take no trips (abl2), against 4:12 and the lean kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06aw}; mkdir -p $O
timeout -k 10 400 python3 -u tools/ab_lookup.py --rounds 9 --only default/lookupN3,ws412/lookupN3,ws412-abl1/lookupN3,ws412-abl2/lookupN3 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail $O/ab.err; exit 1; }
python3 tools/show_ab.py $O/ab.json
