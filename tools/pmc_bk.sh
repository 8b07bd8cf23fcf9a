#!/bin/bash
# PMC passes over the large-batch bucket fold (tools/merge_fold_ab.py --only big), one rocprofv3 run
# per counter group. Usage (GPU box, repo root): tools/pmc_bk.sh OUTDIR
set -u
OUT=${1:-gpurun_out/pmc_bk}
mkdir -p "$OUT"
export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
    "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY" \
    "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
      python3 tools/merge_fold_ab.py --only big --reps 3 ${PMC_BK_ARGS:-} > "$OUT/$tag.log" 2>&1
  rc=$?
  echo "pmc $grp rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; exit $rc; fi
done
