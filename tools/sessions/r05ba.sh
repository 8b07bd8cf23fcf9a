# round 5, call ba: the C2 lookupN(3) bench leg with the library built under other AMDGPU machine
# schedulers (-mllvm -amdgpu-sched-strategy=max-ilp / max-memory-clause / iterative-ilp) against
# the default build, alternating in one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r05ba}; mkdir -p $O
for r in 1 2 3; do
  for v in new max-ilp max-memory-clause iterative-ilp; do
    L=; [ $v != new ] && L=$GRAFT_REPO_ROOT/ringpop-node_amd/ab/librpamd_$v.so
    RP_AMD_LIB=$L timeout -k 10 240 python3 -u bench.py --no-cpu --no-merge --no-wire --no-api --sim-n 0 --sim5-n 0 > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v rc=$?"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"] / 1e9, 2), "G/s", round(d["ms_per_step"], 4), "ms/step", round(d["roofline"].get("kernel_ms", 0) or 0, 4))
PY
  done
done
