#!/bin/bash
# Builds ringpop-node_amd/librpamd_prof.so: the library with the checksum kernel's cycle
# counters compiled in (-DRP_CK_PROF; printf per epoch loop). Load it with RP_AMD_LIB=<path>.
set -e
cd "$(dirname "$0")/../ringpop-node_amd/csrc"
B=${TMPDIR:-/tmp}/rp_profbuild
mkdir -p $B
for f in *.hip; do /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DRP_CK_PROF ${EXTRA:-} -c $f -o $B/${f%.hip}.o & done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../librpamd_prof.so $B/*.o
