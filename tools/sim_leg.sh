#!/bin/bash
# GPU box: the simulator parity tests, then bench.py's C4 + C5 legs only (no CPU legs) under
# rocprofv3 --kernel-trace --stats. Usage (repo root): tools/sim_leg.sh TAG
set -u
TAG=${1:-sim}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_sim_gpu.py tests/test_sim_shard_gpu.py tests/test_sim_digests_gpu.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/test.log" 2>&1
rc=$?; tail -2 "$OUT/test.log"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py \
    --no-cpu --no-merge --no-wire --steps 2 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 - "$OUT" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
for k in ("sim", "sim_c5"):
    v = d.get(k) or {}
    print(k, v.get("ms_per_round"), v.get("rounds_to_convergence"), v.get("round_ms"))
PY
