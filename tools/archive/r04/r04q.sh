# round 4, call q: wire decoder timing ablations (results wrong, times only): abl1 no body name
# lookups, abl2 no record name lookups, abl3 neither; against the in-tree build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q; mkdir -p $O
A=$PWD/ringpop-node_amd/ab
for i in 1 2; do
  for v in tree abl1 abl2 abl3; do
    if [ $v = tree ]; then unset RP_AMD_LIB; else export RP_AMD_LIB=$A/librpamd_$v.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/$v$i.json 2> $O/$v$i.err || { echo "bench $v failed"; tail -20 $O/$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['wire'];print(sys.argv[2], 'enc', round(d['encode']['ms'],3), 'dec', round(d['decode']['ms'],3), d['round_trip_ok'])" $O/$v$i.json $v
  done
done
