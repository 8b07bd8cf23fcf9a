#!/bin/bash
# PMC passes over the membership fold (tools/merge_fold_ab.py) for one library build.
# Usage (GPU box, repo root): tools/pmc_merge.sh OUTDIR [LIB]   (LIB -> RP_AMD_LIB)
# One rocprofv3 run per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -u
OUT=${1:-gpurun_out/pmc_merge}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${2:-}" ]; then export RP_AMD_LIB=$2; fi
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
      python3 tools/merge_fold_ab.py --reps 4 > "$OUT/$tag.log" 2>&1
  rc=$?
  echo "pmc $grp rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; exit $rc; fi
done
