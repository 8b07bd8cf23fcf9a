#!/bin/bash
# GPU box: C5 (one GPU) round time per lane-checksum kernel choice (RP_SIM_CK; "auto" = the
# default choice), bench.py's C5 leg only. Usage (repo root): tools/ck_ab.sh TAG "auto lanes pc32"
set -u
TAG=${1:-ckab}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for v in ${2:-auto lanes pc32}; do
  if [ "$v" = auto ]; then unset RP_SIM_CK; unset RP_SIM_TWINS; else export RP_SIM_CK=$v RP_SIM_TWINS=1; fi
  timeout -k 10 240 python3 -u bench.py --no-cpu --no-merge --no-wire --sim-n 0 \
      --batch-log2 20 --steps 2 --warmup 1 > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v rc=$?"; tail -3 "$OUT/$v.err"; exit 1; }
  python3 - "$OUT/$v.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["sim_c5"]
print(sys.argv[2], round(d["ms_per_round"], 2), d["rounds_to_convergence"], d["round_ms"])
PY
done
