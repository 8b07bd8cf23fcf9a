#!/bin/bash
# GPU box: the default bench line, then the same bench under rocprofv3 --kernel-trace --stats
# (no CPU legs), summaries under gpurun_out/$TAG/. Usage (repo root): tools/bench_prof.sh TAG [bench args]
set -u
TAG=${1:-r02}
shift || true
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
echo "bench ok"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py --no-cpu "$@" \
    > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof rc=$?"; tail -5 "$OUT/prof.err"; exit 1; }
echo "rocprof ok"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -40 "$OUT/kernel_stats.csv" > "$OUT/kernel_top.txt" || true
