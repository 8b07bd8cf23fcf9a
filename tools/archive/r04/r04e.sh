# round 4, call e: the C3 stream length and the checksum slot pool (2 vs 4 groups of 128)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e; mkdir -p $O
for i in 1 2; do
for cfg in "512 1073741824" "512 2147483648" "2048 1073741824" "2048 2147483648"; do
  set -- $cfg
  RP_MEMBERS_CK_BYTES=$2 timeout -k 10 300 python3 -u bench.py --no-cpu --no-api --no-wire --sim-n 0 --sim5-n 0 --steps 2 --warmup 1 --merge-batches $1 > $O/m_$1_$2_$i.json 2> $O/m_$1_$2_$i.err || { echo bench failed; tail -20 $O/m_$1_$2_$i.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['merge'];print(sys.argv[2], round(d['ms_per_batch']*1e3,2), 'us/batch', round(d['updates_per_s']/1e9,3), 'G/s')" $O/m_$1_$2_$i.json "$cfg"
done
done
