"""GPU check of the device sort and scan primitives (rp_prims.hip) that the ring build, the
membership fold and the simulator's inboxes are built on.

rp_selftest_prims (a test-only export, not part of include/ringpop_amd.h) runs the in-place
pair sort, the keys-only sort, the (key, index) sort and both scans on seeded keys and compares
them with std::stable_sort / a host prefix sum: the count of mismatches must be 0 (exact:
stability included). Both the single-pass primitives (decoupled look-back, the default) and the
multi-pass ones (RP_PRIMS_MULTIPASS=1) are checked, across tile boundaries (2048 elements) and
skewed digit distributions.
"""
import ctypes
import json
import os

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SIZES = [0, 1, 2, 2047, 2048, 2049, 6143, 100_000, 1 << 20]
SKEWS = {0: "uniform", 1: "all equal", 2: "16 distinct", 3: "descending"}


def _fn(rpa):
    f = rpa.lib().rp_selftest_prims
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_float)]
    return f


def run(rpa, n, seed, bits, skew, mode, reps=0):
    bad, ms = ctypes.c_uint64(), ctypes.c_float()
    rpa.check(_fn(rpa)(n, seed, bits, skew, mode, reps, ctypes.byref(bad), ctypes.byref(ms)))
    return bad.value, ms.value


@pytest.mark.parametrize("mode", [0, 1], ids=["single-pass", "multi-pass"])
@pytest.mark.parametrize("n", SIZES)
def test_sort_and_scan_exact(rpa, n, mode):
    for bits in (8, 16, 24, 32):
        for skew in SKEWS:
            bad, _ = run(rpa, n, 7 + n + bits, bits, skew, mode)
            assert bad == 0, (n, bits, SKEWS[skew], mode)


def test_large_single_pass(rpa):
    """4M keys (2048 tiles: long look-back chains while the first tiles are still running)."""
    for bits in (24, 32):
        bad, _ = run(rpa, 1 << 22, 99, bits, 0, 0)
        assert bad == 0


def test_single_pass_not_slower(rpa):
    """Device time of the in-place pair sort, single-pass vs multi-pass, written to
    gpurun_out/prims_ab.json; the membership fold's size (1e5 keys, 24 bits) must not be slower."""
    out = {}
    for n, bits in [(100_000, 24), (1 << 20, 32), (1 << 22, 24), (1 << 22, 32)]:
        _, t1 = run(rpa, n, 5, bits, 0, 0, reps=6)
        _, t2 = run(rpa, n, 5, bits, 0, 1, reps=6)
        out["%d/%d" % (n, bits)] = {"single_pass_ms": t1, "multi_pass_ms": t2}
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "prims_ab.json"), "w") as f:
        json.dump(out, f, indent=1)
    r = out["100000/24"]
    assert r["single_pass_ms"] <= r["multi_pass_ms"], out
