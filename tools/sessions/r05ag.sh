# round 5, call ag: bucket fold workgroup size A/B (512 threads kept; ab/librpamd_ft1024.so, ft256), 2^22 in place
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ag; mkdir -p $O
V='{"inplace": {"INPLACE": "1"}}'
for r in 1 2; do
  for v in base ft1024 ft256; do
    L=$PWD/ringpop-node_amd/librpamd.so; [ $v != base ] && L=$PWD/ringpop-node_amd/ab/librpamd_$v.so
    RP_AMD_LIB=$L timeout -k 10 200 python -u tools/ab_fold.py --rounds 8 --out $O/${v}_$r.json --variants "$V" > $O/${v}_$r.log 2>&1 || { echo "ab $v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('$v $r', {k:(v['median_ms'],v['min_ms']) for k,v in d.items()})"
  done
done
