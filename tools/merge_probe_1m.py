"""1M-member table: checksum after the init batch and one C3-shaped batch, on the fold path
RP_MEMBERS_BUCKET_FOLD selects, against the oracle."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import bench  # noqa: E402
import pyoracle  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
torch.cuda.set_device(0)
rpa = bench.load_pkg()
S = bench._synth()
names, st0, inc0 = S.c3_members(n)
m = rpa.Membership(whoami=names[0], capacity=n)
o = pyoracle.Members(names, local=names[0], join_seed=0)
ids0 = np.asarray(m.intern(names), dtype=np.uint32)
a, _, _, na = m.update_ids(ids0, st0, inc0, now_ms=1)
oa, _, _, ona = o.update_ids(ids0, st0, inc0, False, 1)
print("init", na, ona, (a == oa).all(), m.checksum, o.checksum, flush=True)
gs = m.generate_checksum_string()
os_ = o.checksum_string()
print("string len", len(gs), len(os_), gs == os_)
if gs != os_:
    i = next(i for i in range(min(len(gs), len(os_))) if gs[i] != os_[i])
    print("first diff at", i, repr(gs[i - 40:i + 40]), repr(os_[i - 40:i + 40]))
ids, us, ui = S.c3_updates(n, n, seed=41, base_inc=inc0)
ga, _, _, gna = m.update_ids(ids, us, ui, now_ms=1434500000007)
oa, _, _, ona = o.update_ids(ids, us, ui, False, 1434500000007)
print("batch", gna, ona, np.array_equal(ga > 0, oa > 0), m.checksum, o.checksum)
ex, st, inc = m.dump()
bad = [i for i in range(n) if (rpa.STATUS_NAME[int(st[i])], int(inc[i])) != (o.member(names[i])["status"], o.member(names[i])["incarnationNumber"])][:10] if n <= 1 << 16 else None
print("bad rows (small n only)", bad)
