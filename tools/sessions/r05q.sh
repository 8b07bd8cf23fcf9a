# round 5, call q: per-kernel times of the C5 refresh, default against k_ck_tab (RP_SIM_TAB=1), 40 rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05q; mkdir -p $O
for v in base tab; do
  if [ $v = tab ]; then export RP_SIM_TAB=1; else unset RP_SIM_TAB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 -u tools/sim_c5_probe.py 100000 40 > $O/$v.log 2>&1 || { echo "$v failed"; tail -20 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_$v.csv
  t=$(find $O/$v -name "*kernel_trace.csv" | head -1); python3 - $t $v <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "k_ck_" in n or "k_twin" in n or "k_pass1" in n:
        k = n.split("(")[0].split("::")[-1]
        d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(d.items()):
    print(sys.argv[2], k, "n", len(v), "sum %.1f max %.2f" % (sum(v), max(v)), "top", sorted(v)[-6:])
PY
done
grep "round 3[0-9]" $O/base.log | head -3; grep "round 3[0-9]" $O/tab.log | head -3
