#!/bin/bash
# TCP / TA counters of the access-pattern microbenchmark's variants (one launch each, 3 MB table).
set -u
OUT=${1:-gpurun_out/pmc_ub}
mkdir -p "$OUT"
export TMPDIR=/tmp
for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  tag=$(echo $grp | cut -d' ' -f1 )
  timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- ./tools/ub_lookup 5120 q > "$OUT/$tag.log" 2>&1
  echo "pmc $tag rc=$?"
done
