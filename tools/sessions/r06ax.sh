# round 6, call ax: the final checkpoint after the wave-specialised A/B kernel — the full GPU suite, smoke, the default bench line, and the bench
# under rocprofv3 --kernel-trace --stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ax}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/bench_prof.sh r06ax > $O/bench_prof.out 2>&1 || { echo "bench_prof failed"; tail -20 $O/bench_prof.out; exit 1; }
cat $O/bench_prof.out
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"] / 1e9, 2), "G/s ms/step", round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 3))
m = d.get("merge", {})
print("merge", m.get("ms_per_batch"), "fold_large", m.get("fold_large", {}).get("ms_per_batch"))
for k in ("sim", "sim_c5"):
    if k in d: print(k, d[k].get("rounds"), d[k].get("round_ms"))
PY
timeout -k 10 300 python3 -u tools/c5_rounds.py --label default > $O/c5_default.json 2> $O/c5_default.err || { echo "c5 failed"; tail $O/c5_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5_default.json'));ms=[x['ms'] for x in d['per_round']];print('c5 default rounds',d['rounds'],'mean %.1f p50 %.1f p95 %.1f max %.1f'%(sum(ms)/len(ms),d['p50'],d['p95'],max(ms)))"
