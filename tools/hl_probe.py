"""Times rp_hash32_long_dev on a C3-size (3.6 MB) string (with the RP_CK_PROF library it also
prints the chain lane's cycles per chunk)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

rpa = bench.load_pkg()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3_620_017
b = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size=n, dtype=np.uint8)).cuda()
out = torch.zeros(2, dtype=torch.int32, device="cuda")
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rpa.check(rpa.lib().rp_hash32_long_dev(b.data_ptr(), n, out.data_ptr(), None))
    e1.record()
    torch.cuda.synchronize()
    print("hash_long %d bytes: %.3f ms" % (n, e0.elapsed_time(e1)), flush=True)
