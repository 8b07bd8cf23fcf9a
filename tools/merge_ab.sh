#!/bin/bash
# GPU box: the C3 merge leg (bench.py) per checksum group size (RP_MEMBERS_GROUP_SLOTS).
# Usage (repo root): tools/merge_ab.sh TAG "64 128"
set -u
TAG=${1:-mab}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for v in ${2:-64 128}; do
  RP_MEMBERS_GROUP_SLOTS=$v timeout -k 10 240 python3 -u bench.py --no-cpu --no-wire --sim-n 0 --sim5-n 0 \
      --batch-log2 20 --steps 2 --warmup 1 > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v rc=$?"; tail -3 "$OUT/$v.err"; exit 1; }
  python3 - "$OUT/$v.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["merge"]
print(sys.argv[2], round(d["updates_per_s"] / 1e6, 1), "M/s", round(d["ms_per_batch"], 4), "ms/batch", d["checksum"])
PY
done
