"""GPU parity tests of keys grouped by owner through the C ABI (rp_ring_group_keys*):
RingPop.handleOrProxyAll's keysByDest = _.groupBy(keys, this.lookup) (index.js:609-667, :616)
and RequestProxySend.lookupKeys (lib/request-proxy/send.js:171-179).

Oracle: the owners come from oracle/liboracle.so (pinned against the reference's ring goldens in
tests/test_oracle.py); the grouping is underscore's published _.groupBy restated below (walk the
list in order, push onto the owner's array, create it on first sight), and Object.keys order is
insertion order because "host:port" names are never integer-like. Bit-exact.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def ref_group_by(owners):
    """_.groupBy over owner ids: {owner: [key indices]} in first-seen order."""
    out = {}
    for i, o in enumerate(owners):
        out.setdefault(int(o), []).append(i)
    return out


def ring_pair(gpu, orc, n_servers, hash_func=None):
    names = [orc.c2_addr(i) for i in range(n_servers)]
    opts = {"hashFunc": hash_func} if hash_func else None
    ring = gpu.HashRing(opts)
    ring.addRemoveServers(names, names[: n_servers // 10])
    oracle = orc.Ring(100)
    tok = None
    if hash_func:
        tok = np.array([hash_func(s + str(i)) for s in names for i in range(100)], dtype=np.uint32)
    oracle.add_remove(names, names[: n_servers // 10], add_tokens=tok,
                      rem_tokens=None if tok is None else tok[: (n_servers // 10) * 100])
    return ring, oracle


@pytest.mark.parametrize("n_servers,n_keys", [(1, 100), (3, 1000), (64, 10_000), (1000, 50_000)])
def test_group_by_matches_oracle(gpu, orc, n_servers, n_keys):
    ring, oracle = ring_pair(gpu, orc, max(n_servers, 1))
    keys = orc.uuid_keys(42, 0, n_keys)
    want = ref_group_by(oracle.lookup_keys(keys))
    dests, goff, perm = ring.group_ids(keys)
    assert [ring.name(d) for d in dests] == [oracle.name(d) for d in want]
    got = {oracle_id: perm[goff[g]:goff[g + 1]].tolist() for g, oracle_id in enumerate(want)}
    assert got == want
    # the string-level API (keysByDest, lookupKeys)
    skeys = [bytes(k).decode() for k in keys[:2000]]
    kb = ring.groupBy(skeys)
    wb = {}
    for k, o in zip(skeys, oracle.lookup_keys(keys[:2000])):
        wb.setdefault(oracle.name(int(o)), []).append(k)
    assert list(kb.items()) == list(wb.items())
    assert ring.lookupKeys(skeys) == list(wb)


def test_group_by_empty_ring_and_no_keys(gpu):
    ring = gpu.HashRing()
    # lookup's null -> whoami (RingPop.lookup, index.js:434-451): one group, input order
    assert ring.groupBy(["a", "b", "c", "a"], whoami="127.0.0.1:3000") == {"127.0.0.1:3000": ["a", "b", "c", "a"]}
    assert ring.lookupKeys(["x"], whoami="127.0.0.1:3000") == ["127.0.0.1:3000"]
    assert ring.groupBy([]) == {}
    ring.addRemoveServers(["127.0.0.1:3001"], None)
    assert ring.groupBy([]) == {}
    assert ring.groupBy(["k1", "k2"]) == {"127.0.0.1:3001": ["k1", "k2"]}


def test_group_by_hash_func(gpu, orc):
    """options.hashFunc (lib/ring/index.js:29): the caller's key hashes drive the grouping."""
    def hf(s):
        return orc.hash32(s[::-1])

    ring, oracle = ring_pair(gpu, orc, 50, hash_func=hf)
    skeys = ["key-%d" % i for i in range(3000)]
    want = {}
    for k in skeys:
        want.setdefault(oracle.name(oracle.lookup_hash(hf(k))), []).append(k)
    assert list(ring.groupBy(skeys).items()) == list(want.items())


def test_group_dev_large_properties(gpu, orc):
    """2^22 device keys on the C2-shaped ring: the device groups equal the numpy restatement
    over the device owners (themselves pinned by the lookup parity tests), plus the
    size-independent invariants (perm a permutation, groups in first-seen order)."""
    ring, _ = ring_pair(gpu, orc, 10_000)
    n = 1 << 22
    keys = torch.empty(n * 36, dtype=torch.uint8, device="cuda")
    gpu.gen_uuid_keys_dev(42, 0, n, keys.data_ptr())
    own = torch.empty(n, dtype=torch.int32, device="cuda")
    ring.lookup_dev(keys.data_ptr(), n, own.data_ptr())
    dests = torch.empty(n, dtype=torch.int32, device="cuda")
    goff = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    perm = torch.empty(n, dtype=torch.int32, device="cuda")
    nd = torch.zeros(1, dtype=torch.int32, device="cuda")
    ring.group_dev(keys.data_ptr(), n, dests.data_ptr(), goff.data_ptr(), perm.data_ptr(), nd.data_ptr())
    torch.cuda.synchronize()
    o = own.cpu().numpy().view(np.uint32)
    k = int(nd.item())
    uniq, first = np.unique(o, return_index=True)
    order = np.argsort(first, kind="stable")
    assert k == len(uniq)
    assert (dests[:k].cpu().numpy().view(np.uint32) == uniq[order]).all()
    rank = np.empty(int(uniq.max()) + 1, dtype=np.int64)
    rank[uniq[order]] = np.arange(k)
    want_perm = np.argsort(rank[o], kind="stable")
    assert (perm.cpu().numpy() == want_perm).all()
    cnt = np.bincount(rank[o], minlength=k)
    assert (goff[: k + 1].cpu().numpy() == np.concatenate([[0], np.cumsum(cnt)])).all()
