"""GPU parity tests of the device hash ring through the C ABI (librpamd.so).

Oracles: tests/golden/ring_golden.json (what the reference JS returned, lib/ring/index.js +
rbtree.js) and oracle/liboracle.so (the CPU restatement, pinned against those goldens in
tests/test_oracle.py). Integer/index work: every comparison is bit-exact.
"""
import random

import numpy as np
import pytest

import golden_util as gu

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def names_to_idx(ring, ids, names):
    return [-1 if x == 0xFFFFFFFF else names.index(ring.name(x)) for x in ids]


@pytest.mark.parametrize("case_name", ["c1", "collide", "port", "port1", "tiny"])
def test_ring_matches_reference_goldens(gpu, orc, case_name):
    case = next(c for c in gu.load("ring_golden.json")["cases"] if c["name"] == case_name)
    hf = gu.hash_func(case)
    opts = {"replicaPoints": case["replicaPoints"]}
    if hf is not None:
        opts["hashFunc"] = hf
    ring = gpu.HashRing(opts)
    names = case["names"]
    assert ring.checksum is None  # hashring_test.js:95-99
    for b in case["batches"]:
        changed = ring.addRemoveServers(b["add"], b["remove"])
        assert changed == b["changed"]
        assert ring.getServerCount() == b["serverCount"]
        assert list(ring.servers) == b["servers"]  # Object.keys(ring.servers), insertion order
        assert ring.getStats()["servers"] == b["servers"]
        assert sorted(ring.name(i) for i in ring.server_ids()) == sorted(b["servers"])  # the device's set
        assert ring.size == b["size"]
        assert ring.checksum == b["checksum"]
        if "tree" in b:
            t, o = ring.dump()
            assert t.tolist() == b["tree"]["tokens"]
            assert names_to_idx(ring, o, names) == b["tree"]["owners"]
        if "keys" not in b:
            continue
        keys = gu.keys_of(b)
        assert names_to_idx(ring, ring.lookup_ids(keys), names) == b["lookup"]
        for n, lists in b["lookupN"].items():
            ids, cnt = ring.lookupn_ids(keys, int(n))
            got = [names_to_idx(ring, row[:c], names) for row, c in zip(ids, cnt)]
            assert got == lists, "lookupN n=%s" % n


def test_reference_ring_test_1000_lookups(gpu):
    # test/unit/ring-test.js:66-80 — lookup(server + '0') === server with the real hash
    servers = ["127.0.0.1:%d" % (3000 + i) for i in range(1000)]
    ring = gpu.HashRing()
    ring.addRemoveServers(servers, None)
    assert ring.getServerCount() == 1000
    got = ring.lookup_ids([s + "0" for s in servers])
    assert [ring.name(x) for x in got] == servers
    ring.addRemoveServers(None, servers)  # ring-test.js:38-51
    assert ring.getServerCount() == 0
    ring.addRemoveServers(servers, servers)
    assert ring.getServerCount() == 0
    assert ring.lookup("anything") is None
    assert ring.lookupN("anything", 3) == []


def test_hashring_events_and_checksum_order_independence(gpu):
    # test/unit/hashring_test.js:51-166
    r1, r2 = gpu.HashRing(), gpu.HashRing()
    ev = []
    r1.on("added", lambda n: ev.append(("a", n))).on("removed", lambda n: ev.append(("r", n)))
    for i in range(4):
        r1.addServer("127.0.0.1:300%d" % i)
    for i in reversed(range(4)):
        r2.addServer("127.0.0.1:300%d" % i)
    assert r1.checksum == r2.checksum is not None
    assert r1.size == 400
    c0 = r1.checksum
    r1.removeServer("127.0.0.1:3001")
    r1.removeServer("127.0.0.1:3001")  # no-op: absent
    assert ev.count(("r", "127.0.0.1:3001")) == 1
    assert r1.checksum != c0 and r1.size == 300
    r3 = gpu.HashRing()
    r3.removeServer("127.0.0.1:3000")
    assert r3.checksum is None  # hashring_test.js:101-105
    r4 = gpu.HashRing({"replicaPoints": 200})
    r4.addServer("test 1")
    assert r4.size == 200 and r4.servers == {"test 1": True}


def _random_history(orc, gpu, seed, pool_size, R, nbatches):
    rng = random.Random(seed)
    pool = [orc.c2_addr(i * 7 + seed) for i in range(pool_size)]
    ring, oracle = gpu.HashRing({"replicaPoints": R}), orc.Ring(R)
    for _ in range(nbatches):
        add = rng.sample(pool, rng.randint(0, pool_size // 2))
        rem = rng.sample(pool, rng.randint(0, pool_size // 3))
        assert ring.addRemoveServers(add, rem) == oracle.add_remove(add, rem)
        assert ring.checksum == oracle.checksum
        t, o = ring.dump()
        ot, oo = oracle.dump()
        assert np.array_equal(t, ot)
        assert [ring.name(x) for x in o] == [oracle.name(x) for x in oo]
    return ring, oracle


# lookup layouts/kernels (rp_ring.hip): compact = the default C2 hot path (k_lookupn_lean, 8 keys
# per lane staged in four slices for lookupN(3));
# round1 = k_lookupn_compact over the same layout; window = the packed probe kernel; packed / wide = the generic kernels over those layouts.
LAYOUTS = {
    "compact": {},
    "compact-kpl1": {"RP_LOOKUP_KPL": "1"},
    "compact-kpl2": {"RP_LOOKUP_KPL": "2"},
    "compact-kpl3": {"RP_LOOKUP_KPL": "3"},
    "compact-kpl8": {"RP_LOOKUP_KPL": "8"},
    "half": {"RP_LOOKUP_HALF": "2"},
    "half-kpl2": {"RP_LOOKUP_HALF": "2", "RP_LOOKUP_KPL": "2"},
    "half-kpl8": {"RP_LOOKUP_HALF": "2", "RP_LOOKUP_KPL": "8"},
    "quarter-kpl8": {"RP_LOOKUP_HALF": "4", "RP_LOOKUP_KPL": "8"},
    # three workgroups striding over every tile (RP_LOOKUP_GRID): LDS lists and counters reused
    "quarter-kpl8-grid3": {"RP_LOOKUP_HALF": "4", "RP_LOOKUP_KPL": "8", "RP_LOOKUP_GRID": "3"},
    # deferred keys finished by the lean kernel's own workgroups (no k_lookupn_fix_tiles)
    "fusefix": {"RP_LOOKUP_FUSEFIX": "1"},
    "fusefix-grid3": {"RP_LOOKUP_FUSEFIX": "1", "RP_LOOKUP_GRID": "3"},
    # key slices DMA'd global -> LDS (global_load_lds_dwordx4) through a two-buffer ring
    "stg1": {"RP_LOOKUP_STG": "1"},
    "stg1-grid3": {"RP_LOOKUP_STG": "1", "RP_LOOKUP_GRID": "3"},
    "stg1-lh2": {"RP_LOOKUP_STG": "1", "RP_LOOKUP_LH": "2"},
    "lh2": {"RP_LOOKUP_LH": "2"},
    # the same DMA issued from asm (no compiler drain before the slice reads): 8 or 4 key slices,
    # lookups in two halves or all at once
    "stg2": {"RP_LOOKUP_STG": "2"},
    "stg2-grid3": {"RP_LOOKUP_STG": "2", "RP_LOOKUP_GRID": "3"},
    "stg2-lh1": {"RP_LOOKUP_STG": "2", "RP_LOOKUP_LH": "1"},
    "stg2-hs4": {"RP_LOOKUP_STG": "2", "RP_LOOKUP_STGHS": "4"},
    # window 1 at the bucket start (the round-2 placement) instead of the predicted start
    "wpred0": {"RP_LOOKUP_WPRED": "0"},
    # lookupN(3) without the hinted index (the round-4 index and window start)
    "hint0": {"RP_LOOKUP_HINT": "0"},
    "lean-kpl4": {"RP_LOOKUP_HALF": "0", "RP_LOOKUP_KPL": "4"},
    "round1": {"RP_LOOKUP_LEAN": "0"},
    "round1-kpl1": {"RP_LOOKUP_LEAN": "0", "RP_LOOKUP_KPL": "1"},
    "window": {"RP_RING_LAYOUT": "packed"},
    "packed": {"RP_RING_LAYOUT": "packed", "RP_RING_NOWINDOW": "1"},
    "wide": {"RP_RING_WIDE": "1"},
    # the LDS-index kernel (round 6, k_lookupn_lds): the bucket index in every CU's LDS, one L2 trip
    # a key; "lds-grid3": three workgroups striding every wave-tile
    "lds": {"RP_LOOKUP_LDS": "1"},
    "lds-grid3": {"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_GRID": "3"},
    "lean": {"RP_LOOKUP_LDS": "0"},
    # the wave-specialised kernel (round 6, k_lookupn_ws): producer waves stream and hash the keys
    # into an LDS ring, consumer waves take the index and window trips; NP:NC waves a workgroup,
    # "ws-grid1": one workgroup through every wave-tile (the ring's slots reused many times)
    "ws": {"RP_LOOKUP_WS": "1:3"},
    "ws-2-6": {"RP_LOOKUP_WS": "2:6"},
    "ws-1-7": {"RP_LOOKUP_WS": "1:7"},
    "ws-4-12": {"RP_LOOKUP_WS": "4:12"},
    "ws-2-2": {"RP_LOOKUP_WS": "2:2"},
    "ws-1-15": {"RP_LOOKUP_WS": "1:15"},
    "ws-2-14": {"RP_LOOKUP_WS": "2:14"},
    "ws-grid1": {"RP_LOOKUP_WS": "1:3", "RP_LOOKUP_WS_GRID": "1"},
}


def set_layout(monkeypatch, layout):
    for k in ("RP_RING_WIDE", "RP_RING_NOWINDOW", "RP_RING_LAYOUT", "RP_LOOKUP_KPL", "RP_LOOKUP_LEAN", "RP_LOOKUP_HALF",
              "RP_LOOKUP_GRID", "RP_LOOKUP_FUSEFIX", "RP_LOOKUP_WPRED", "RP_LOOKUP_STG", "RP_LOOKUP_LH",
              "RP_LOOKUP_STGHS", "RP_LOOKUP_HINT", "RP_LOOKUP_LDS", "RP_LOOKUP_LDS_GRID", "RP_LOOKUP_WS",
              "RP_LOOKUP_WS_GRID"):
        monkeypatch.delenv(k, raising=False)
    if layout != "compact" and not layout.startswith("lds"):  # every other layout names a lean / older kernel
        monkeypatch.setenv("RP_LOOKUP_LDS", "0")
    for k, v in LAYOUTS[layout].items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("layout", list(LAYOUTS))
def test_random_histories_vs_oracle(gpu, orc, layout, monkeypatch):
    set_layout(monkeypatch, layout)
    ring, oracle = _random_history(orc, gpu, 3, 300, 100, 12)
    keys = orc.uuid_keys(99, 0, 20000)
    want = oracle.lookup_keys(keys)
    got = ring.lookup_ids(keys)
    assert [ring.name(x) for x in got] == [oracle.name(x) for x in want]
    for n in (-1, 0, 1, 2, 3, 4, 5, 8, 9, 17):
        w, wc = oracle.lookupn_keys(keys[:3000], n)
        g, gc = ring.lookupn_ids(keys[:3000], n)
        assert np.array_equal(gc, wc), n
        for row_g, row_w, c in zip(g, w, wc):
            assert [ring.name(x) for x in row_g[:c]] == [oracle.name(x) for x in row_w[:c]]
            assert (row_g[c:] == 0xFFFFFFFF).all()


def test_variable_length_keys_vs_oracle(gpu, orc):
    ring, oracle = _random_history(orc, gpu, 8, 50, 100, 2)
    rng = random.Random(1)
    keys = ["".join(rng.choice("abcdef0123456789:-./") for _ in range(rng.randint(0, 70))) for _ in range(5000)]
    keys += [str(i) for i in range(200)] + ["", "x" * 1000]
    hs = [orc.hash32(k) for k in keys]
    want = [oracle.lookup_hash(h) for h in hs]
    got = ring.lookup_ids(keys)
    assert [ring.name(x) for x in got] == [oracle.name(x) for x in want]
    g, gc = ring.lookupn_ids(keys, 3)
    for k, (row, c) in enumerate(zip(g, gc)):
        assert [ring.name(x) for x in row[:c]] == [oracle.name(x) for x in oracle.lookupn_hash(hs[k], 3)]


@pytest.mark.parametrize("nkeys", [1, 7, 64, 65])
def test_small_host_batches_vs_oracle(gpu, orc, nkeys, monkeypatch):
    """The one-call drop-in path: host batches of at most 64 keys (3 KB) and 16 owners per row
    go through the kernel arguments and pinned memory (k_lookupn_small); 65 keys, a 3,100-byte
    key or wider rows take the staged path. Both against the oracle, lookup and lookupN(n) for
    n = 0..20."""
    ring, oracle = _random_history(orc, gpu, 8, 50, 100, 3)
    rng = random.Random(nkeys)
    keys = ["".join(rng.choice("abcdef0123456789:-./") for _ in range(rng.randint(0, 45))) for _ in range(nkeys)]
    if nkeys == 7:
        keys[3] = "y" * 3100  # past the inline bytes: the staged path
    hs = [orc.hash32(k) for k in keys]
    got = ring.lookup_ids(keys)
    assert [ring.name(x) for x in got] == [oracle.name(oracle.lookup_hash(h)) for h in hs]
    for n in (0, 1, 2, 3, 8, 9, 16, 17, 20):
        g, gc = ring.lookupn_ids(keys, n)
        for k, (row, c) in enumerate(zip(g, gc)):
            assert [ring.name(x) for x in row[:c]] == [oracle.name(x) for x in oracle.lookupn_hash(hs[k], n)], (n, k)
    monkeypatch.setenv("RP_RING_SMALL", "0")
    g0, c0 = ring.lookupn_ids(keys, 3)
    monkeypatch.delenv("RP_RING_SMALL")
    g1, c1 = ring.lookupn_ids(keys, 3)
    assert np.array_equal(g0, g1) and np.array_equal(c0, c1)


@pytest.mark.parametrize("svc", ["2", "2-nodt", "2-w1", "2-ans0", "1"],
                         ids=["v3", "v3-window", "v3-one-wave", "v3-lds-answer", "round4"])
def test_lookup_service_vs_oracle(gpu, orc, svc, monkeypatch):
    """The resident lookup service (rp_ring_service): one-key lookup / lookupN calls through
    pinned host lines, against the oracle, for key lengths 0..180 (1-3 key lines; longer keys
    and n > 8 take the small path), across a ring mutation (which stops the service and rebuilds
    the table it reads), an idle exit (the next call relaunches it) and turning it off. "v3":
    the host-hashed service with its direct table (few servers: the successor lists are
    complete) and its kSvcWaves pollers answering each request, some more than once;
    "v3-window": RP_SVC_DT=0, the compact window and walks; "v3-one-wave": RP_SVC_WAVES=1;
    "v3-lds-answer": RP_SVC_ANS=0, the round-5 record answer (LDS slots, duplicate scan)."""
    if svc.endswith("-nodt"):
        monkeypatch.setenv("RP_SVC_DT", "0")
        svc = svc[:-5]
    if svc.endswith("-w1"):
        monkeypatch.setenv("RP_SVC_WAVES", "1")
        svc = svc[:-3]
    if svc.endswith("-ans0"):
        monkeypatch.setenv("RP_SVC_ANS", "0")
        svc = svc[:-5]
    import time
    ring, oracle = _random_history(orc, gpu, 8, 50, 100, 3)
    rng = random.Random(77)
    keys = ["".join(rng.choice("abcdef0123456789:-./") for _ in range(L)) for L in
            list(range(0, 70)) + [119, 120, 121, 179, 180, 181, 300]]
    hs = [orc.hash32(k) for k in keys]
    monkeypatch.setenv("RP_RING_SVC", svc)  # read by ring.service()
    ring.service(50)

    def check_all(r, o):
        for k, h in zip(keys, hs):
            assert [r.name(x) for x in r.lookup_ids([k])] == [o.name(o.lookup_hash(h))], k
            for n in (0, 1, 3, 8, 9):
                g, gc = r.lookupn_ids([k], n)
                assert [r.name(x) for x in g[0][:gc[0]]] == [o.name(x) for x in o.lookupn_hash(h, n)], (n, k)

    check_all(ring, oracle)
    extra = ["svc-%d:3000" % i for i in range(5)]
    ring.addRemoveServers(extra, [])
    oracle.add_remove(extra, [])
    check_all(ring, oracle)
    time.sleep(0.2)  # past the 50 ms idle exit
    check_all(ring, oracle)
    ring.service(0)
    check_all(ring, oracle)


@pytest.mark.parametrize("dt", ["1", "0"], ids=["direct", "window"])
def test_lookup_service_c2_vs_oracle(gpu, orc, monkeypatch, dt):
    """The service on the C2 ring (10k servers x 100 points): 3,000 single-key lookup and
    lookupN(1..8) calls with 36-byte UUID keys against the oracle. "direct": one 64-B record of
    the direct table per key (k_dt_build; 2^20 buckets); "window": RP_SVC_DT=0, the compact
    layout's two-trip window (svc_compact_window, n <= 4) and the exact walks."""
    monkeypatch.setenv("RP_SVC_DT", dt)
    servers = c2_servers(orc, 10000)
    ring = gpu.HashRing()
    ring.addRemoveServers(servers)
    oracle = orc.Ring(100)
    oracle.add_remove(servers)
    keys = [k.tobytes().decode() for k in orc.uuid_keys(7, 0, 3000)]
    ring.service(200)
    for i, k in enumerate(keys):
        h = orc.hash32(k)
        n = 1 + i % 8
        g, gc = ring.lookupn_ids([k], n)
        assert [ring.name(x) for x in g[0][:gc[0]]] == [oracle.name(x) for x in oracle.lookupn_hash(h, n)], (i, k)
        if i % 10 == 0:
            assert [ring.name(x) for x in ring.lookup_ids([k])] == [oracle.name(oracle.lookup_hash(h))]
        if i % 10 == 5:  # a caller hash (hashFunc) through the service
            g, gc = ring.lookupn_hashes([h ^ 0x5bd1e995], n)
            assert [ring.name(x) for x in g[0][:gc[0]]] == \
                [oracle.name(x) for x in oracle.lookupn_hash(h ^ 0x5bd1e995, n)], (i, k)
    # keys past the round-4 kernel's 180 bytes go through the service too
    for L in (181, 500, 4000):
        k = "x" * L
        h = orc.hash32(k)
        assert [ring.name(x) for x in ring.lookup_ids([k])] == [oracle.name(oracle.lookup_hash(h))]
    ring.service(0)


def test_lookup_service_direct_table_collisions(gpu, orc):
    """The direct table where it cannot answer alone: a caller hashFunc with few distinct values
    (hash32 % 257: about half the buckets hold more than 7 equal tokens and overflow their record,
    the others answer from it; equal tokens keep the ring's order), 40 servers x 50 points; lookupN(1..8) and lookup of 600 keys
    through the service against the oracle with the same tokens (the record, or the fallback
    paths when it overflows)."""
    servers = ["dt-%d:3000" % i for i in range(40)]
    R = 50

    def hf(s):
        return orc.hash32(s) % 257 * 16711433 & 0xFFFFFFFF

    ring = gpu.HashRing({"replicaPoints": R, "hashFunc": hf})
    ring.addRemoveServers(servers)
    oracle = orc.Ring(R)
    oracle.add_remove(servers, [], [hf(s + str(i)) for s in servers for i in range(R)], None)
    ring.service(200)
    rng = random.Random(11)
    for i in range(600):
        h = rng.getrandbits(32) if i % 3 else hf("key-%d" % i)
        n = 1 + i % 8
        g, gc = ring.lookupn_hashes([h], n)
        assert [ring.name(x) for x in g[0][:gc[0]]] == [oracle.name(x) for x in oracle.lookupn_hash(h, n)], (i, h, n)
    ring.service(0)


def test_lookup_service_then_growing_batch(gpu, orc):
    """A batch lookup after service lookups does not wait for the service wave to idle out
    (ADVICE r4): with idle_ms = 3000, single-key lookups leave the wave resident; a batch larger
    than any before (its staging buffers grow: hipFree synchronizes the device) must return well
    under idle_ms, because every non-service ring path stops the service first. Results against
    the oracle."""
    import time
    ring, oracle = _random_history(orc, gpu, 8, 50, 100, 3)
    ring.service(3000)
    rng = random.Random(5)
    keys = ["k%d-%s" % (i, rng.random()) for i in range(40)]
    for k in keys[:8]:
        assert [ring.name(x) for x in ring.lookup_ids([k])] == [oracle.name(oracle.lookup_hash(orc.hash32(k)))]
    big = ["b%d" % i for i in range(200000)]
    t0 = time.perf_counter()
    g, gc = ring.lookupn_ids(big, 3)
    dt = time.perf_counter() - t0
    assert dt < 1.5, dt
    hs = [orc.hash32(k) for k in big[:2000]]
    for row, c, h in zip(g[:2000], gc[:2000], hs):
        assert [ring.name(x) for x in row[:c]] == [oracle.name(x) for x in oracle.lookupn_hash(h, 3)]
    # the service comes back for the next single call
    assert [ring.name(x) for x in ring.lookup_ids([keys[9]])] == [oracle.name(oracle.lookup_hash(orc.hash32(keys[9])))]
    ring.service(0)


def test_lookup_service_beside_growing_membership(gpu, orc):
    """a resident service must not stall another handle. A ring with
    service(3000) answers single-key lookups from a thread every ~2 ms (the per-request
    RingPop.lookup of handleOrProxy, index.js:434-451) while a Membership in the same process
    applies batches of new members whose buffers grow 10 -> 10k -> 100k (gossip's update,
    lib/on_membership_event.js:106-134: both in one process). Before the QuietScope every
    buffer growth (hipFree) waited for the wave, which the lookups kept resident for up to its
    30 s lifetime. Each update and checksum read must return in < 50 ms; the updates equal the
    oracle's, the lookups the ring oracle's."""
    import threading
    import time
    servers = ["svc-m-%d:3000" % i for i in range(64)]
    ring, roracle = gpu.HashRing(), orc.Ring(100)
    ring.addRemoveServers(servers)
    roracle.add_remove(servers)
    keys = ["req-%d" % i for i in range(512)]
    want = [roracle.name(roracle.lookup_hash(orc.hash32(k))) for k in keys]
    ring.service(3000)
    n = 110_000
    names = ["10.%d.%d.%d:3000" % (i >> 16, (i >> 8) & 255, i & 255) for i in range(n)]
    # warm the membership kernels (first-launch code object loads) before any timing
    w = gpu.Membership(whoami=names[0])
    w.update_ids(w.intern(names[:20]), [0] * 20, [5] * 20, now_ms=1)
    _ = w.checksum
    w.close()

    stop = threading.Event()
    log = {"n": 0, "bad": [], "lat": []}

    def lookups():
        i = 0
        while not stop.is_set():
            t0 = time.perf_counter()
            got = ring.name(ring.lookup_ids([keys[i % len(keys)]])[0])
            log["lat"].append(time.perf_counter() - t0)
            if got != want[i % len(keys)]:
                log["bad"].append(i)
            log["n"] += 1
            i += 1
            time.sleep(0.002)

    m = gpu.Membership(whoami=names[0], capacity=16)
    o = orc.Members(names, local=names[0])
    th = threading.Thread(target=lookups, daemon=True)
    th.start()
    try:
        lo = 0
        rng = np.random.default_rng(3)
        for step, hi in enumerate((10, 10_000, 100_000, n)):
            # new members (the table, names and checksum buffers grow) plus updates of known ones
            ids_new = np.arange(lo, hi, dtype=np.uint32)
            ids_old = rng.integers(0, max(lo, 1), size=(hi - lo) // 4, dtype=np.uint32)
            ids = np.concatenate([ids_new, ids_old])
            st = rng.integers(0, 4, size=len(ids), dtype=np.uint8)
            inc = rng.integers(1, 4, size=len(ids), dtype=np.int64)
            dev_ids = np.asarray(m.intern([names[i] for i in ids]), dtype=np.uint32)
            ring.lookup_ids([keys[step]])  # the service wave is resident as the update starts
            t0 = time.perf_counter()
            ga, gs, gi, gna = m.update_ids(dev_ids, st, inc, now_ms=100 + step)
            t_up = time.perf_counter() - t0
            t0 = time.perf_counter()
            ck = m.checksum
            t_ck = time.perf_counter() - t0
            oa, os_, oi, ona = o.update_ids(ids, st, inc, False, 100 + step)
            assert gna == ona and np.array_equal(ga > 0, oa > 0), step
            assert np.array_equal(gs[oa > 0], os_[oa > 0]) and np.array_equal(gi[oa > 0], oi[oa > 0])
            assert ck == o.checksum, step
            assert t_up < 0.05 and t_ck < 0.05, (step, hi, t_up, t_ck)
            lo = hi
    finally:
        stop.set()
        th.join(10)
    assert not log["bad"] and log["n"] >= 10, log["n"]
    assert max(log["lat"]) < 0.5, max(log["lat"])
    ring.service(0)
    m.close()
    ring.close()


def test_device_farmhash_and_keygen(gpu, orc):
    rng = random.Random(2)
    strs = [bytes(rng.randrange(256) for _ in range(n)) for n in list(range(0, 80)) * 3 + [500, 4096]]
    blob = b"".join(strs)
    off = np.zeros(len(strs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in strs])
    d_b = torch.tensor(list(blob) + [0], dtype=torch.uint8, device="cuda")
    d_o = torch.from_numpy(off.view(np.int64)).cuda()
    d_out = torch.empty(len(strs), dtype=torch.int32, device="cuda")
    gpu.check(gpu.lib().rp_hash32_batch_dev(d_b.data_ptr(), d_o.data_ptr(), len(strs), d_out.data_ptr(), None))
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint32)
    assert got.tolist() == [orc.hash32(s) for s in strs]
    n = 100003
    d_k = torch.empty(n * 36, dtype=torch.uint8, device="cuda")
    gpu.gen_uuid_keys_dev(42, 12345, n, d_k.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(d_k.cpu().numpy().reshape(n, 36), orc.uuid_keys(42, 12345, n))


@pytest.mark.parametrize("pack", ["1", "0"], ids=["pack16", "one-per-workgroup"])
def test_long_hash_multi_vs_oracle(gpu, orc, pack, monkeypatch):
    """rp_hash32_long_multi_dev (the membership checksum groups' chains): 41 strings side by side,
    lengths 0..1.3 MB (the <= 24-byte forms, every 20-byte chunk boundary near 25..65, long ones
    of different lengths in one workgroup, so the packed kernel's lockstep part stops at the
    shortest and the rest run masked), some gated off (left untouched), against the oracle's
    farmhash32. "pack16": k_hash_long_pack, 16 strings a workgroup (round 6); the other: one
    workgroup a string."""
    monkeypatch.setenv("RP_HL_PACK", pack)
    rng = np.random.default_rng(9)
    lens = [0, 1, 4, 5, 12, 13, 24, 25, 26, 44, 45, 46, 64, 65, 66, 100, 1000, 4096, 20000, 100003,
            1_300_000, 1_299_981, 1_299_999, 777_777, 65, 3, 2_000, 60_001, 45, 1_000_000, 999_990,
            25, 250_000, 24, 400_019, 17, 1_234_567, 88, 9_999, 1_048_576, 31]
    gate = [0 if i % 7 == 5 else 1 for i in range(len(lens))]
    stride = ((max(lens) + 32 + 255) // 256) * 256
    buf = rng.integers(32, 127, size=stride * len(lens), dtype=np.uint8)
    meta = np.zeros(4 * len(lens), dtype=np.uint32)
    meta[0::4] = np.asarray(lens, dtype=np.uint32) + 1
    meta[1::4] = gate
    meta[2::4] = 0xDEADBEEF
    d_b = torch.from_numpy(buf).cuda()
    d_m = torch.from_numpy(meta.view(np.int32)).cuda()
    gpu.check(gpu.lib().rp_hash32_long_multi_dev(d_b.data_ptr(), stride, len(lens), d_m.data_ptr(), None))
    torch.cuda.synchronize()
    got = d_m.cpu().numpy().view(np.uint32).reshape(-1, 4)
    for b, (L, g) in enumerate(zip(lens, gate)):
        if g:
            assert (got[b, 2], got[b, 3]) == (orc.hash32(buf[b * stride:b * stride + L].tobytes()), 1), (b, L)
        else:
            assert (got[b, 2], got[b, 3]) == (0xDEADBEEF, 0), (b, L)


def c2_servers(orc, n):
    return [orc.c2_addr(i) for i in range(n)]


@pytest.mark.parametrize("layout", list(LAYOUTS))
def test_device_resident_lookupn_c1_vs_oracle(gpu, orc, layout, monkeypatch):
    set_layout(monkeypatch, layout)
    # C1 shape (1000 servers x 100 points), 1M device-generated keys, lookup + lookupN(3)
    servers = gu.load("ring_golden.json")["cases"][0]["batches"][0]["add"]
    ring, oracle = gpu.HashRing(), orc.Ring(100)
    ring.addRemoveServers(servers)
    oracle.add_remove(servers)
    n = 1 << 20
    d_k = torch.empty(n * 36, dtype=torch.uint8, device="cuda")
    gpu.gen_uuid_keys_dev(42, 0, n, d_k.data_ptr())
    d_o = torch.empty(n * 3, dtype=torch.int32, device="cuda")
    d_c = torch.empty(n, dtype=torch.uint8, device="cuda")
    ring.lookupn_dev(d_k.data_ptr(), n, 3, d_o.data_ptr(), d_c.data_ptr())
    d_l = torch.empty(n, dtype=torch.int32, device="cuda")
    ring.lookup_dev(d_k.data_ptr(), n, d_l.data_ptr())
    torch.cuda.synchronize()
    keys = orc.uuid_keys(42, 0, n)
    w, wc = oracle.lookupn_keys(keys, 3, threads=8)
    # ids are interned in the same first-seen order on both sides for a single add batch
    assert np.array_equal(d_o.cpu().numpy().view(np.uint32).reshape(n, 3), w)
    assert np.array_equal(d_c.cpu().numpy(), wc)
    assert np.array_equal(d_l.cpu().numpy().view(np.uint32), w[:, 0])


_C2_OWNERS = {}


def _c2_oracle_owners(orc, oracle, n):
    """The oracle's lookupN(key, 3) owners of the first n C2 keys (seed 42), computed once."""
    if n not in _C2_OWNERS:
        keys = orc.uuid_keys(42, 0, n)
        _C2_OWNERS[n] = oracle.lookupn_keys(keys, 3, threads=16)[0]
        del keys
    return _C2_OWNERS[n]


@pytest.mark.parametrize("layout", ["compact", "round1", "lean-kpl4", "half-kpl8", "fusefix", "wpred0", "stg2", "stg1", "hint0",
                                    "lds", "lean", "ws", "ws-2-6", "ws-1-7", "ws-4-12", "ws-2-2", "ws-1-15", "ws-2-14"])
def test_c2_full_size_properties(gpu, orc, layout, monkeypatch):
    set_layout(monkeypatch, layout)
    # C2: 10k servers x 100 points (~1M tokens); 2^24 keys on device; size-independent
    # properties at full size, and every key's owners equal to the oracle's.
    servers = c2_servers(orc, 10000)
    ring = gpu.HashRing()
    ring.addRemoveServers(servers)
    oracle = orc.Ring(100)
    oracle.add_remove(servers)
    assert ring.checksum == oracle.checksum
    assert ring.size == oracle.token_count()
    t, o = ring.dump()
    assert (np.diff(t.astype(np.int64)) > 0).all()  # sorted, unique
    n = 1 << 24
    d_k = torch.empty(n * 36, dtype=torch.uint8, device="cuda")
    gpu.gen_uuid_keys_dev(42, 0, n, d_k.data_ptr())
    d_o = torch.empty(n * 3, dtype=torch.int32, device="cuda")
    d_c = torch.empty(n, dtype=torch.uint8, device="cuda")
    ring.lookupn_dev(d_k.data_ptr(), n, 3, d_o.data_ptr(), d_c.data_ptr())
    torch.cuda.synchronize()
    own = d_o.cpu().numpy().view(np.uint32).reshape(n, 3)
    assert (d_c.cpu().numpy() == 3).all()
    assert (own < 10000).all()
    assert ((own[:, 0] != own[:, 1]) & (own[:, 1] != own[:, 2]) & (own[:, 0] != own[:, 2])).all()
    # load balance sanity: every server owns some keys
    assert np.bincount(own[:, 0], minlength=10000).min() > 0
    # exact on all 2^24 keys (round 4; 2^21 before): the oracle's answer is computed once for
    # every layout (fingerprint ties, long buckets and the ring end all occur)
    w = _c2_oracle_owners(orc, oracle, n)
    assert np.array_equal(own, w)
    d_l = torch.empty(n, dtype=torch.int32, device="cuda")
    ring.lookup_dev(d_k.data_ptr(), n, d_l.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(d_l.cpu().numpy().view(np.uint32), w[:, 0])


def test_edge_cases(gpu):
    ring = gpu.HashRing()
    assert ring.lookup("k") is None and ring.lookupN("k", 3) == [] and ring.lookupN("k", 0) == []
    ring.addServer("only")
    assert ring.lookupN("k", 3) == ["only"]  # ring-test.js:102-116 (size 1)
    assert ring.lookupN("k", 0) in (["only"], [])
    assert ring.lookupN("k", -5) == ring.lookupN("k", 0)
    assert ring.lookup("k") == "only"
    ids, cnt = ring.lookupn_ids([], 3)
    assert len(ids) == 0 and len(cnt) == 0


@pytest.mark.parametrize("layout", ["compact", "compact-kpl1", "compact-kpl3", "compact-kpl8", "round1",
                                    "round1-kpl1", "half", "half-kpl2", "half-kpl8", "quarter-kpl8", "lean-kpl4", "window",
                                    "fusefix", "wpred0", "stg2", "stg2-hs4", "ws", "ws-4-12", "ws-grid1"])
@pytest.mark.parametrize("nserv,R", [(1, 100), (2, 2000), (3, 700), (5, 5), (40, 1), (64, 3)])
def test_window_kernel_slow_paths_vs_oracle(gpu, orc, nserv, R, layout, monkeypatch):
    """Rings that force the window kernels' exact fallbacks: long buckets, runs of one owner,
    wrap past the last token, rings smaller than the window."""
    set_layout(monkeypatch, layout)
    servers = [orc.c2_addr(i + 17) for i in range(nserv)]
    ring, oracle = gpu.HashRing({"replicaPoints": R}), orc.Ring(R)
    ring.addRemoveServers(servers)
    oracle.add_remove(servers)
    n = (1 << 16) + 77  # a partial last tile goes through the generic kernel
    d_k = torch.empty(n * 36, dtype=torch.uint8, device="cuda")
    gpu.gen_uuid_keys_dev(5, 0, n, d_k.data_ptr())
    keys = orc.uuid_keys(5, 0, n)
    for nrep in (-1, 0, 1, 2, 3, 4):
        w = max(nrep, 1)
        d_o = torch.empty(n * w, dtype=torch.int32, device="cuda")
        d_c = torch.empty(n, dtype=torch.uint8, device="cuda")
        ring.lookupn_dev(d_k.data_ptr(), n, nrep, d_o.data_ptr(), d_c.data_ptr())
        torch.cuda.synchronize()
        want, wc = oracle.lookupn_keys(keys, nrep)
        got = d_o.cpu().numpy().view(np.uint32).reshape(n, w)
        assert np.array_equal(d_c.cpu().numpy(), wc), nrep
        assert np.array_equal(got, want), nrep


@pytest.mark.parametrize("length", [0, 7, 24, 25, 44, 45, 164, 165, 20 * 1024 + 1, 20 * 1024 + 20,
                                    20 * 1024 * 3 + 7, 100_003, 3_620_017])
def test_device_long_hash_vs_oracle(gpu, orc, length):
    """rp_hash32_long_dev (the checksum strings' serial chain, k_hash_long) at lengths around
    the 20-byte chunk, the 8-chunk unroll and the 1024-chunk LDS window boundaries."""
    rng = np.random.default_rng(length)
    b = rng.integers(0, 256, size=length + 1, dtype=np.uint8)
    d = torch.from_numpy(b).cuda()
    out = torch.zeros(2, dtype=torch.int32, device="cuda")
    gpu.check(gpu.lib().rp_hash32_long_dev(d.data_ptr(), length, out.data_ptr(), None))
    torch.cuda.synchronize()
    assert int(out.cpu().numpy().view(np.uint32)[0]) == orc.hash32(bytes(b[:length]))


@pytest.mark.parametrize("servers,R,mod", [(1, 1, 0), (2, 3, 0), (3, 50, 0), (5, 7, 97), (17, 20, 0), (40, 100, 65521)])
def test_lookup_service_direct_table_small_rings(gpu, orc, servers, R, mod):
    """The service's direct table on small rings (fewer distinct owners than its 16 successor
    slots: the records carry the complete flag), with and without colliding caller tokens:
    lookupN(1..8) of 400 hashes each (random, at token values, one past them, 0 and 2^32 - 1)
    against the oracle."""
    names = ["s%d:%d" % (i, 3000 + i) for i in range(servers)]

    def hf(s):
        h = orc.hash32(s)
        return (h % mod) * 65537 & 0xFFFFFFFF if mod else h

    ring = gpu.HashRing({"replicaPoints": R, "hashFunc": hf})
    ring.addRemoveServers(names)
    oracle = orc.Ring(R)
    toks = [hf(s + str(i)) for s in names for i in range(R)]
    oracle.add_remove(names, [], toks, None)
    ring.service(200)
    rng = random.Random(servers * 1000 + R)
    hs = [0, 0xFFFFFFFF] + [t for t in toks[:60]] + [(t + 1) & 0xFFFFFFFF for t in toks[:60]]
    hs += [rng.getrandbits(32) for _ in range(400 - len(hs))]
    for i, h in enumerate(hs):
        n = 1 + i % 8
        g, gc = ring.lookupn_hashes([h], n)
        assert [ring.name(x) for x in g[0][:gc[0]]] == [oracle.name(x) for x in oracle.lookupn_hash(h, n)], (i, h, n)
    ring.service(0)
