# round 5, call s: C5 refresh kernel times: k_ck_lanes / k_ck_tab 8 KB window (2 workgroups a CU) /
# k_ck_tab 16 KB window (ab/librpamd_tab16k.so, one workgroup a CU); simulator tests on the 16 KB build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s; mkdir -p $O
RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_tab16k.so RP_SIM_TAB=1 timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py -k "tab" > $O/tests16k.log 2>&1 || { echo tests failed; tail -40 $O/tests16k.log; exit 1; }
tail -1 $O/tests16k.log
for v in base tab tab16k; do
  case $v in base) unset RP_SIM_TAB; L=$PWD/ringpop-node_amd/librpamd.so;; tab) export RP_SIM_TAB=1; L=$PWD/ringpop-node_amd/librpamd.so;; tab16k) export RP_SIM_TAB=1; L=$PWD/ringpop-node_amd/ab/librpamd_tab16k.so;; esac
  RP_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python3 -u tools/sim_c5_probe.py 100000 40 > $O/$v.log 2>&1 || { echo "$v failed"; tail -20 $O/$v.log; exit 1; }
done
python3 - $O <<'PY'
import csv, re, collections, sys, glob
for v in ("base", "tab", "tab16k"):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(glob.glob(sys.argv[1] + "/" + v + "/*kernel_trace.csv")[0])):
        m = re.search(r"(k_ck_\w+)", r["Kernel_Name"])
        if m:
            d[m.group(1)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, x in sorted(d.items()):
        print(v, k, "n", len(x), "sum %.1f max %.2f" % (sum(x), max(x)), [round(y, 1) for y in sorted(x)[-6:]])
PY
