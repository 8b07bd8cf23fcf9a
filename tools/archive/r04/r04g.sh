# round 4, call g: k_ck_lanes without the per-group register copy (loop unrolled by two):
# simulator goldens + C4/C5 digests, then C4/C5 bench legs against the previous library
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests/test_sim_gpu.py tests/test_sim_digests_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for lib in ringpop-node_amd/ab/librpamd_simbase.so ringpop-node_amd/librpamd.so; do
    RP_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu --no-api --no-wire --no-merge --steps 2 --warmup 1 > $O/sim_$(basename $lib .so)_$i.json 2> $O/sim_$(basename $lib .so)_$i.err || { echo bench failed; tail -20 $O/sim_$(basename $lib .so)_$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['sim_c5'];c4=d['sim'];print(sys.argv[2], 'C4', round(c4['ms_per_round'],2), 'C5', round(c['ms_per_round'],2), c['round_ms'])" $O/sim_$(basename $lib .so)_$i.json $(basename $lib .so)
  done
done
