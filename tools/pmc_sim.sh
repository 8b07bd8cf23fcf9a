#!/bin/bash
# PMC passes for the simulator's checksum kernels on a C4-size run (GPU box, repo root).
set -u
OUT=${1:-gpurun_out/pmc_sim}
N=${2:-20000}
mkdir -p "$OUT"
export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
  tag=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
      python3 tools/sim_probe.py $N 1 60 > "$OUT/$tag.log" 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; exit $rc; fi
done
