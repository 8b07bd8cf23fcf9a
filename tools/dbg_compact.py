import os, sys, torch
sys.path.insert(0, "/root/repo")
import bench
rpa = bench.load_pkg()
os.environ["RP_LOOKUP_DEBUG"] = "1"
for S in (1000, 10000):
    ring = rpa.HashRing()
    ring.addRemoveServers([bench.c2_addr(i) for i in range(S)])
    B = 1 << 22
    keys = torch.empty(B * 36, dtype=torch.uint8, device="cuda")
    rpa.gen_uuid_keys_dev(42, 0, B, keys.data_ptr())
    out = torch.empty(B * 3, dtype=torch.int32, device="cuda")
    ring.lookupn_dev(keys.data_ptr(), B, 3, out.data_ptr())
    torch.cuda.synchronize()
