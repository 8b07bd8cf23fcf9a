"""A/B of the 2^22 bucket fold's kernel variants in ONE process (round 5): one table of 2^22
members, fresh 2^22-update batches (checksum deferred, as bench.py's fold_large), the variants'
environment knobs switched batch by batch in rotation, HIP events per batch.

    python tools/ab_fold.py --variants '{"new": {}, "old": {"RP_BK_REC8": "0"}, "inplace": {"INPLACE": "1"}}' [--rounds 6]

(INPLACE=1: the status / incarnation outputs alias the inputs, as the reference rewrites its
update objects in place; otherwise separate output arrays.)

Prints per variant the median / min ms per batch and the fraction of 8 TB/s at 49 B per update.
"""
import argparse
import importlib.util
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNOBS = ("RP_BK_DIRECT", "RP_BK_REC8", "RP_BK_SGRID")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--log2", type=int, default=22)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    variants = json.loads(a.variants)
    import torch
    rpa = _load("ringpop_node_amd", os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    n = k = 1 << a.log2
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    m = rpa.Membership(whoami=names[0], capacity=n)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, np.zeros(n, np.uint8), inc0, now_ms=1)
    rpa.check(rpa.lib().rp_members_defer_checksum(m._h, 1))
    nsets = 3
    sets = []
    for q in range(nsets):
        ids, us, ui = S.c3_updates(n, k, seed=300 + q, base_inc=inc0 + 3 * q)
        sets.append((torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(),
                     torch.from_numpy(ui).cuda()))
    app = torch.empty(k, dtype=torch.uint8, device="cuda")
    nst = torch.empty(k, dtype=torch.uint8, device="cuda")
    ninc = torch.empty(k, dtype=torch.int64, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")
    nb = [0]

    def one(inplace):
        b = nb[0]
        nb[0] += 1
        d = sets[b % nsets]
        inc = d[2] + 3 * nsets * (b // nsets)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        os_, oi = (d[1], inc) if inplace else (nst, ninc)  # in place: the outputs are the inputs
        m.update_dev(d[0].data_ptr(), d[1].data_ptr(), inc.data_ptr(), k, 1434500000000 + b, app.data_ptr(),
                     os_.data_ptr(), oi.data_ptr(), na.data_ptr(), sp)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), int(na.item())

    times = {v: [] for v in variants}
    for r in range(a.rounds + 1):
        for name, env in variants.items():
            for kn in KNOBS:
                os.environ.pop(kn, None)
            os.environ.update({x: v for x, v in env.items() if x != "INPLACE"})
            ms, napp = one(env.get("INPLACE") == "1")
            if r:
                times[name].append(ms)
        print("round %d done (applied %d)" % (r, napp), flush=True)
    res = {}
    for name, t in times.items():
        med = float(np.median(t))
        res[name] = {"env": variants[name], "median_ms": round(med, 4), "min_ms": round(float(np.min(t)), 4),
                     "frac_49B": round(49 * k / (med * 1e-3) / 1e9 / 8000, 4)}
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    m.close()


if __name__ == "__main__":
    main()
