"""CPU tests of the C ABI: librpamd.so builds, loads without a GPU, exports every symbol the
public header declares, and its host farmhash32 agrees with the oracle (no device calls)."""
import os
import random
import re

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(REPO, "include", "ringpop_amd.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(rpa):
    L = rpa.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    # and the Python binding types every one of them
    assert set(syms) == set(rpa.SIGNATURES)


def test_version_and_no_device_is_not_a_crash(rpa):
    assert rpa.lib().rp_version() >> 16 == 1
    assert rpa.device_count() >= 0


def test_host_farmhash_matches_oracle_all_length_classes(rpa, orc):
    rng = random.Random(5)
    cases = [b"", b"a", b"ab", b"abc", b"abcd", b"\xff\x80", bytes(range(256))]
    for n in list(range(0, 90)) + [100, 255, 1000, 4097]:
        for _ in range(5):
            cases.append(bytes(rng.randrange(256) for _ in range(n)))
    for c in cases:
        assert rpa.hash32(c) == orc.hash32(c), (len(c), c[:16])
    assert rpa.hash32("") == 0xDC56D17A


def test_host_farmhash_replica_strings(rpa, orc):
    for s in ["10.28.5.35:20800", "127.0.0.1:3000", "test 1"]:
        for i in range(120):
            assert rpa.hash32(s + str(i)) == orc.hash32(s + str(i))
