#!/bin/bash
# SQ (instruction-issue) PMC passes for the compact lookupN kernel (GPU box, repo root): is the
# kernel VALU-issue bound, L2-request bound or waiting? One --pmc pass per group.
set -u
OUT=${1:-gpurun_out/pmc_sq}
VARIANTS=${2:-compact-kpl4/lookupN3}
mkdir -p "$OUT"
export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CU_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  tag=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
      python3 tools/ab_lookup.py --rounds 2 --only "$VARIANTS" > "$OUT/$tag.log" 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; exit $rc; fi
done
