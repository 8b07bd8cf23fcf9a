# round 5, call ah: the refresh kernel choice threshold (RP_SIM_PC32_PER_CU: k_ck_pc<3,2> when the dirty
# views fill at most that many 64-view groups per CU, else k_ck_lanes), C4/C5 bench legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ah; mkdir -p $O
for i in 1 2; do
  for v in 3 2 4 6; do
    RP_SIM_PC32_PER_CU=$v timeout -k 10 300 python3 -u bench.py --no-cpu --no-api --no-wire --no-merge --steps 2 --warmup 1 > $O/pc${v}_$i.json 2> $O/pc${v}_$i.err || { echo bench failed; tail -20 $O/pc${v}_$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['sim_c5'];c4=d['sim'];print('pc', sys.argv[2], 'C4', round(c4['ms_per_round'],2), 'C5', round(c['ms_per_round'],2), {k: round(x,1) if isinstance(x,float) else x for k,x in c['round_ms'].items()})" $O/pc${v}_$i.json $v
  done
done
