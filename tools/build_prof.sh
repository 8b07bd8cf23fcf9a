#!/bin/bash
# Builds a diagnostics copy of the library with cycle counters compiled in. Load it with
# RP_AMD_LIB=<path>.
#   tools/build_prof.sh              -> librpamd_prof.so   (-DRP_CK_PROF: checksum chain epochs)
#   DEFS=-DRP_LK_PROF OUT=librpamd_lkprof.so tools/build_prof.sh   (lean lookup phases)
#   DEFS=-DRP_LK_ABLATE OUT=librpamd_lkabl.so tools/build_prof.sh (RP_LOOKUP_ABLATE timing ablations)
set -e
cd "$(dirname "$0")/../ringpop-node_amd/csrc"
DEFS=${DEFS:--DRP_CK_PROF}
OUT=${OUT:-librpamd_prof.so}
B=${TMPDIR:-/tmp}/rp_profbuild_${OUT%.so}
mkdir -p $B
for f in *.hip; do /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $DEFS ${EXTRA:-} -c $f -o $B/${f%.hip}.o & done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../$OUT $B/*.o
