"""Synthetic inputs of SURVEY.md §8d (numpy, vectorised Philox4x32-10).

The reference draws ids and timing from Math.random / uuid.v4; every workload here is a
deterministic function of (seed, counter) so the device, the CPU oracle and the injected
reference harness see identical inputs. Philox4x32-10 is checked against the oracle's C
implementation and the Random123 known answers in tests/test_synth.py.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)

TAG_MEMBER = 0x4D454D42  # 'MEMB'
TAG_UPDATE = 0x55504454  # 'UPDT'
BASE_INC = 1434401518824  # benchmarks/large-membership.json's first incarnation number


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays (counters) and scalar keys."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32).copy() for x in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0), np.uint32(k1)
    for _ in range(10):
        p0 = M0 * c0.astype(np.uint64)
        p1 = M1 * c2.astype(np.uint64)
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK).astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def stream(seed, tag, n, start=0):
    ctr = np.arange(start, start + n, dtype=np.uint64)
    lo = (ctr & MASK).astype(np.uint32)
    hi = (ctr >> np.uint64(32)).astype(np.uint32)
    z = np.zeros(n, dtype=np.uint32)
    return philox4x32_10(lo, hi, z, z, seed, tag)


def c2_addr(i):
    """SURVEY §8d C2/C3 address of member/server i."""
    return "10.%d.%d.%d:%d" % ((i >> 16) & 255, (i >> 8) & 255, i & 255, 20800 + i % 36)


def c3_members(n, seed=7):
    """C3 member table: addresses c2_addr(i), all alive, inc = BASE_INC + philox(i) % 10^8."""
    r0, _, _, _ = stream(seed, TAG_MEMBER, n)
    inc = np.int64(BASE_INC) + (r0.astype(np.int64) % np.int64(10 ** 8))
    return [c2_addr(i) for i in range(n)], np.zeros(n, dtype=np.uint8), inc


def c3_updates(n_members, k, seed=7, base_inc=None):
    """C3 update batch: ids visit a permutation of the members, 1% of records repeat an earlier
    record's address (order-sensitive fold); status ~ {alive .70, suspect .15, faulty .10,
    leave .05}; inc = the member's base incarnation + {-1, 0, +1}."""
    if base_inc is None:
        base_inc = c3_members(n_members, seed)[2]
    r0, r1, r2, r3 = stream(seed, TAG_UPDATE, k)
    j = np.arange(k, dtype=np.int64)
    ids = ((7919 * j + 12345) % n_members).astype(np.int64)
    dup = (r0 % 100 == 0) & (j > 0)
    src = (r1.astype(np.int64) % np.maximum(j, 1))
    # a duplicate copies the id of an earlier record (resolved in order: chains allowed)
    for q in np.nonzero(dup)[0]:
        ids[q] = ids[src[q]]
    u = r2 % 100
    status = np.where(u < 70, 0, np.where(u < 85, 1, np.where(u < 95, 2, 3))).astype(np.uint8)
    inc = base_inc[ids] + (r3.astype(np.int64) % 3) - 1
    return ids.astype(np.uint32), status, inc.astype(np.int64)


TAG_KILL = 0x4B494C4C  # 'KILL'
NOW0 = BASE_INC + 10 ** 9  # Date.now() at round 0 of the gossip model (+200 ms per round)


def kill_set(n, k, seed=11):
    """the k members killed before round 0 (partial Fisher-Yates over a
    Philox stream); returns a uint8 mask of length n."""
    perm = np.arange(n, dtype=np.int64)
    r = stream(seed, TAG_KILL, max(k, 1))[0]
    for i in range(k):
        j = i + int((int(r[i]) * (n - i)) >> 32)
        perm[i], perm[j] = perm[j], perm[i]
    dead = np.zeros(n, dtype=np.uint8)
    dead[perm[:k]] = 1
    return dead
