# round 4, call h: the chain kernels' rare paths out of line (k_ck_lanes 78 -> 27 KB of code):
# A = round-3 loop + noinline, B = loop unrolled by two + noinline; sim parity on both, then
# C4/C5 legs against the round-3 library
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h; mkdir -p $O
for v in A B; do
RP_AMD_LIB=ringpop-node_amd/ab/librpamd_sim$v.so timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests/test_sim_gpu.py tests/test_sim_digests_gpu.py > $O/tests_$v.log 2>&1 || { echo tests $v failed; tail -40 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
for i in 1 2; do
  for lib in simbase simA simB; do
    RP_AMD_LIB=ringpop-node_amd/ab/librpamd_$lib.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-api --no-wire --no-merge --steps 2 --warmup 1 > $O/sim_${lib}_$i.json 2> $O/sim_${lib}_$i.err || { echo bench failed; tail -20 $O/sim_${lib}_$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['sim_c5'];c4=d['sim'];print(sys.argv[2], 'C4', round(c4['ms_per_round'],2), 'C5', round(c['ms_per_round'],2), {k:round(v,1) for k,v in c['round_ms'].items()})" $O/sim_${lib}_$i.json $lib
  done
done
