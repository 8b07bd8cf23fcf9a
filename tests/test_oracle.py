"""CPU tests: the oracle is pinned against published known answers and against the golden
vectors the reference JS produced (tests/golden/ring_golden.json)."""
import re

import numpy as np
import pytest

import golden_util as gu


def test_farmhash_published_known_answer(orc):
    # FarmHash / go-farm published value: Hash32("") == Fingerprint32("") == 0xdc56d17a
    assert orc.hash32("") == 0xDC56D17A


def test_philox_random123_kat(orc):
    assert orc.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert orc.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert orc.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_uuid_key_format(orc):
    keys = orc.uuid_keys(42, 0, 1000)
    pat = re.compile(rb"^[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}$")
    for k in keys:
        assert pat.match(k.tobytes())
    assert len({k.tobytes() for k in keys}) == 1000
    # stream is positional: keys [500, 1000) == stream started at 500
    assert np.array_equal(orc.uuid_keys(42, 500, 500), keys[500:])


def test_c2_addr(orc):
    assert orc.c2_addr(0) == "10.0.0.0:20800"
    assert orc.c2_addr(70000) == "10.1.17.112:20816"


def _replay_oracle(orc, case):
    R = case["replicaPoints"]
    hf = gu.hash_func(case)
    names = case["names"]
    ring = orc.Ring(R)
    for b in case["batches"]:
        at = rt = None
        if hf is not None:
            at = [hf(s + str(i)) for s in b["add"] for i in range(R)]
            rt = [hf(s + str(i)) for s in b["remove"] for i in range(R)]
        yield ring, b, ring.add_remove(b["add"], b["remove"], at, rt), hf, names


@pytest.mark.parametrize("case_name", ["c1", "collide", "port", "port1", "tiny"])
def test_oracle_matches_reference_ring(orc, case_name):
    case = next(c for c in gu.load("ring_golden.json")["cases"] if c["name"] == case_name)
    for ring, b, changed, hf, names in _replay_oracle(orc, case):
        assert changed == b["changed"]
        assert ring.server_count() == b["serverCount"]
        assert ring.token_count() == b["size"]
        if hf is None:
            assert ring.checksum == b["checksum"]
        t, o = ring.dump()
        if "tree" in b:
            assert list(t) == b["tree"]["tokens"]
            assert [names.index(ring.name(x)) for x in o] == b["tree"]["owners"]
        if "keys" not in b:
            continue
        keys = gu.keys_of(b)
        hs = [hf(k) if hf else orc.hash32(k) for k in keys]
        got = [-1 if (x := ring.lookup_hash(h)) == orc.NIL else names.index(ring.name(x)) for h in hs]
        assert got == b["lookup"]
        for n, lists in b["lookupN"].items():
            got = [[names.index(ring.name(x)) for x in ring.lookupn_hash(h, int(n))] for h in hs]
            assert got == lists, "lookupN n=%s" % n


def test_ring_ops_golden_inherited_names(orc):
    """tests/golden/ring_ops_golden.json (reference single calls with names the servers map
    inherits, e.g. 'constructor'): after every call the ring equals the oracle ring of the listed
    own servers (checksum, token count); inherited names never own a token."""
    for case in gu.load("ring_ops_golden.json")["cases"]:
        R = case["replicaPoints"]
        for op, r in zip(case["ops"], case["results"]):
            ring = orc.Ring(R)
            ring.add_remove(r["servers"], [])
            assert ring.checksum == r["checksum"], op
            assert ring.token_count() == r["size"] == R * r["serverCount"], op
        rets = [r["ret"] for r in case["results"]]
        assert rets[3] is None and "removed:constructor" in case["results"][3]["events"]
        assert rets[4] is False and rets[5] is True
