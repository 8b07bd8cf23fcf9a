#!/bin/bash
# SQ counters of the simulator's checksum kernels over the first C5 rounds (GPU box, repo root):
# VALU / LDS instruction counts, LDS bank-conflict cycles and the waves' busy cycles.
set -u
OUT=${1:-gpurun_out/pmc_ck}
R=${2:-12}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA"; do
  tag=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "k_ck_" --output-format csv -d "$OUT/$tag" -o run -- \
      python3 tools/sim_c5_probe.py 100000 $R > "$OUT/$tag.log" 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; exit $rc; fi
done
