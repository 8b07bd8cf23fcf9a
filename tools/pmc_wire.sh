#!/bin/bash
# PMC passes for the wire decoder's wave kernel on the bench's wire leg (GPU box, repo root).
# Summarise with tools/pmc_wire_summary.py <out dir>.
set -u
OUT=${1:-gpurun_out/pmc_wire}
mkdir -p "$OUT"
export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
  tag=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
      python3 bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 1 --warmup 0 --batch-log2 20 > "$OUT/$tag.log" 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; exit $rc; fi
done
