"""Phase cycle counters of the lean lookupN kernel on the C2 ring (diagnostics).

    DEFS=-DRP_LK_PROF OUT=librpamd_lkprof.so tools/build_prof.sh
    RP_AMD_LIB=ringpop-node_amd/librpamd_lkprof.so RP_LK_PROF_PRINT=1 python tools/lk_phase.py

Runs 40 launches of lookupN(3) over 2^26 keys (the bench's workload); the library prints, per
launch, the cycles a wave spends per tile in each phase (summed over waves / wave-tiles).
Extra environment knobs (RP_LOOKUP_*) pass through.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    rpa = bench.load_pkg()
    ring = rpa.HashRing()
    ring.addRemoveServers([bench.c2_addr(i) for i in range(10000)])
    B = 1 << 26
    st = torch.cuda.current_stream()
    keys = torch.empty(B * 36, dtype=torch.uint8, device="cuda")
    rpa.gen_uuid_keys_dev(42, 0, B, keys.data_ptr(), st.cuda_stream)
    out = torch.empty(B * 3, dtype=torch.int32, device="cuda")
    n = int(os.environ.get("LK_N", "3"))
    for i in range(int(os.environ.get("LK_LAUNCHES", "40"))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        ring.lookupn_dev(keys.data_ptr(), B, n, out.data_ptr(), None, 36, None, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        print("launch %d: %.4f ms" % (i, e0.elapsed_time(e1)), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
