# round 5, call p: the refresh over shared pre-mix tables (k_ck_tab, RP_SIM_TAB=1): simulator kernel
# tests, then C4/C5 bench legs alternating with the default refresh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py -k "tab or lanes" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in base tab; do
    if [ $v = tab ]; then export RP_SIM_TAB=1; else unset RP_SIM_TAB; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu --no-api --no-wire --no-merge --steps 2 --warmup 1 > $O/sim_${v}_$i.json 2> $O/sim_${v}_$i.err || { echo bench failed; tail -20 $O/sim_${v}_$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['sim_c5'];c4=d['sim'];print(sys.argv[2], 'C4', round(c4['ms_per_round'],2), 'C5', round(c['ms_per_round'],2), c['round_ms'], c.get('rounds'), c.get('checksum_digest', c.get('digest')))" $O/sim_${v}_$i.json $v
  done
done
