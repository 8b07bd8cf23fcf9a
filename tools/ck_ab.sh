#!/bin/bash
# GPU box: C4 and C5 (one GPU) round times per checksum-kernel choice, bench.py's sim legs only.
# Variants: auto (defaults), d1blk (RP_SIM_D1_BLOCKCK=1: ping-req senders' checksums by one
# workgroup each inside D1), lanes / pc32 / pc (RP_SIM_CK, twins on).
# Usage (repo root): tools/ck_ab.sh TAG "auto hw0"
set -u
TAG=${1:-ckab}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for v in ${2:-auto hw0}; do
  unset RP_SIM_CK RP_SIM_TWINS RP_SIM_HW RP_SIM_D1_BLOCKCK RP_SIM_PC32_PER_CU
  case $v in
    auto) ;;
    hw0) export RP_SIM_HW=0 ;;
    d1blk) export RP_SIM_D1_BLOCKCK=1 ;;
    cu2) export RP_SIM_PC32_PER_CU=2 ;;
    cu4) export RP_SIM_PC32_PER_CU=4 ;;
    cu6) export RP_SIM_PC32_PER_CU=6 ;;
    *) export RP_SIM_CK=$v RP_SIM_TWINS=1 ;;
  esac
  timeout -k 10 240 python3 -u bench.py --no-cpu --no-merge --no-wire \
      --batch-log2 20 --steps 2 --warmup 1 > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v rc=$?"; tail -3 "$OUT/$v.err"; exit 1; }
  python3 - "$OUT/$v.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("sim", "sim_c5"):
    s = d[k]
    print(sys.argv[2], k, round(s["ms_per_round"], 3), s["rounds_to_convergence"], {q: round(x, 1) if isinstance(x, float) else x for q, x in s["round_ms"].items()})
PY
done
