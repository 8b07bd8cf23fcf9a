# round 5, call am: k_ck_lanes2 (two views per lane, 128 views a wave): simulator kernel tests, then
# C4/C5 bench legs alternating with the default refresh, and the refresh kernels' times over 40 C5 rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05am; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py -k "lanes2" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in base l2; do
    if [ $v = l2 ]; then export RP_SIM_LANES2=1; else unset RP_SIM_LANES2; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu --no-api --no-wire --no-merge --steps 2 --warmup 1 > $O/sim_${v}_$i.json 2> $O/sim_${v}_$i.err || { echo bench failed; tail -20 $O/sim_${v}_$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['sim_c5'];c4=d['sim'];print(sys.argv[2], 'C4', round(c4['ms_per_round'],2), 'C5', round(c['ms_per_round'],2), {k: round(x,1) if isinstance(x,float) else x for k,x in c['round_ms'].items()}, c.get('rounds'))" $O/sim_${v}_$i.json $v
  done
done
export RP_SIM_LANES2=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/l2 -o run -- python3 -u tools/sim_c5_probe.py 100000 40 > $O/l2.log 2>&1 || { echo "prof failed"; tail -20 $O/l2.log; exit 1; }
python3 - $O <<'PY'
import csv, re, collections, sys, glob
d = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(sys.argv[1] + "/l2/*kernel_trace.csv")[0])):
    m = re.search(r"(k_ck_\w+)", r["Kernel_Name"])
    if m:
        d[m.group(1)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, x in sorted(d.items()):
    print("l2", k, "n", len(x), "sum %.1f max %.2f" % (sum(x), max(x)), [round(y, 1) for y in sorted(x)[-6:]])
PY
rm -rf $O/l2
