"""numpy emulation of the LDS-index lookup layout (k_lidx_build / k_lpack3 / k_lookupn_lds,
rp_ring.hip) on the C2 ring: checks that every key the kernel would resolve in its window gets the
oracle's lookupN(3) owners, and prints why the others are deferred (fingerprint ties, groups with
a bucket of 16+ tokens, a window that misses, the ring end), for window offsets d = 2..5.

    python tools/emu_lds.py [--keys 2000000]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle as orc  # noqa: E402

U = np.uint64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=2_000_000)
    ap.add_argument("--check", type=int, default=200_000)
    a = ap.parse_args()
    o = orc.Ring(100)
    o.add_remove([orc.c2_addr(i) for i in range(10000)])
    tok, own = o.dump()
    tok, own = tok.astype(U), own.astype(U)
    M = len(tok)
    lg = 6
    while lg < 13 and (1 << lg) * 126 < M:
        lg += 1
    ng, ob = 1 << lg, 14
    fb = 24 - ob
    t = ((tok << U(lg)) & U(0xFFFFFFFF)) * U(28)
    bt = (tok >> U(32 - lg)) * U(28) + (t >> U(32))
    cnt = np.bincount(bt.astype(np.int64), minlength=ng * 28)
    start = np.concatenate([[0], np.cumsum(cnt)])
    full_g = (cnt.reshape(ng, 28) > 15).any(1)
    pred = (np.arange(ng, dtype=U) * U(M)) >> U(lg)
    delta = start[np.arange(ng) * 28].astype(np.int64) - pred.astype(np.int64)
    print("M %d lg %d: delta %d..%d, max tokens a bucket %d, groups with a bucket of 16+ %d"
          % (M, lg, delta.min(), delta.max(), cnt.max(), full_g.sum()))
    ent = np.concatenate([(((t & U(0xFFFFFFFF)) >> U(32 - fb)) << U(ob)) | own, np.full(40, 0xFFFFFF, U)])
    h = np.random.default_rng(5).integers(0, 2 ** 32, size=a.keys, dtype=U)
    pos = np.searchsorted(tok, h, side="left")
    th = ((h << U(lg)) & U(0xFFFFFFFF)) * U(28)
    gh = (h >> U(32 - lg)).astype(np.int64)
    b = gh * 28 + (th >> U(32)).astype(np.int64)
    fr = th & U(0xFFFFFFFF)
    c = cnt[b]
    st = start[b]
    fl = (((fr >> U(24)) * c.astype(U)) >> U(8)).astype(np.int64)
    K = (fr >> U(32 - fb)) << U(ob)
    om = U((1 << ob) - 1)

    def exact3(p):
        out, j = [], p % M
        while len(out) < 3:
            if own[j] not in out:
                out.append(own[j])
            j = (j + 1) % M
        return out

    for d in (2, 3, 4, 5):
        s = np.maximum(fl - d, 0)
        w0 = st + s
        e = ent[np.clip(w0[:, None] + np.arange(10)[None, :], 0, len(ent) - 1)]
        inb = (s[:, None] + np.arange(10)[None, :]) < c[:, None]
        lt = (inb & (e < K[:, None])).sum(1)
        diff = e.astype(np.int64) - K[:, None].astype(np.int64)
        tie = (inb & (diff >= 0) & (diff < (1 << ob))).any(1)
        under, end = (s > 0) & (lt == 0), w0 + 12 > M
        slow = tie | full_g[gh] | under | (lt == 10) | end
        bad = nchk = short = 0
        for i in np.nonzero(~slow)[0][:a.check]:
            out = []
            for j in range(lt[i], 10):
                if (e[i, j] & om) not in out:
                    out.append(e[i, j] & om)
                if len(out) == 3:
                    break
            if len(out) < 3:
                short += 1
                continue
            nchk += 1
            bad += out != exact3(pos[i])
        print("d=%d deferred %.3f%% (tie %.3f, full group %.3f, before window %.3f, past %.4f, end %.4f, "
              "owners short %d); checked %d, wrong %d"
              % (d, 100 * slow.mean(), 100 * tie.mean(), 100 * full_g[gh].mean(), 100 * under.mean(),
                 100 * (lt == 10).mean(), 100 * end.mean(), short, nchk, bad))


if __name__ == "__main__":
    main()
