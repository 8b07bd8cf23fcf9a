#!/bin/bash
# PMC passes for the lookupN kernels (run on the GPU box from the repo root).
# Separate passes per counter group (guide: FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -u
OUT=${1:-gpurun_out/pmc}
VARIANTS=${2:-window/lookupN3,packed/lookupN3}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
      python3 tools/ab_lookup.py --rounds 2 --only "$VARIANTS" > "$OUT/$tag.log" 2>&1
  rc=$?
  echo "pmc $grp rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
