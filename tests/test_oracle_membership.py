"""CPU tests: the membership oracle (oracle/orc_members.c) reproduces what the reference
Membership (lib/membership/*.js) did on every golden op: applied updates (incl. the local
override rewrite), member order (injected getJoinPosition), checksum and checksum string."""
import pytest

import golden_util as gu

STAT = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}


def case_names(case):
    seen = {case["local"]: None}
    for op in case["ops"]:
        for ch in op.get("changes", []):
            seen.setdefault(ch[0], None)
    return list(seen)


def replay(orc, case):
    m = orc.Members(case_names(case), local=case["local"], join_seed=case["joinSeed"])
    for op in case["ops"]:
        if op["type"] == "ready":
            m.set_ready(op["value"])
        elif op["type"] == "set":
            m.set()
        else:
            ch = op["changes"]
            app, nst, ninc, _ = m.update_ids([m.index[c[0]] for c in ch], [STAT[c[1]] for c in ch],
                                             [c[2] for c in ch], op.get("isLocal", False), op.get("now", 0))
            got = [[i, orc.STATUS_NAME[int(nst[i])], int(ninc[i])] for i in range(len(ch)) if app[i]]
            yield op, got, m
            continue
        yield op, None, m


@pytest.mark.parametrize("case_name", ["random", "fixture1332", "stash-set", "leave", "rules"])
def test_membership_oracle_matches_reference(orc, case_name):
    cases = gu.load("membership_golden.json")["cases"]
    sel = [c for c in cases if c["name"].startswith("rule/")] if case_name == "rules" else \
        [c for c in cases if c["name"] == case_name]
    assert sel
    for case in sel:
        for op, got, m in replay(orc, case):
            if got is not None:
                assert got == op["applied"], (case["name"], op.get("now"))
            assert m.checksum == op["checksum"], case["name"]
            if "members" in op:
                want = op["members"]
                assert m.order() == [w[0] for w in want], case["name"]
                assert [[a, m.member(a)["status"], m.member(a)["incarnationNumber"]] for a in m.order()] == want
            if isinstance(op.get("checksumString"), str):
                assert m.checksum_string() == op["checksumString"]


def test_member_order_independent_of_read_schedule(orc):
    """The oracle places joined members lazily (a log of splice positions resolved by a Fenwick
    tree when the order is read, round 5): the members array must come out the same whether it
    is read after every batch or once at the end, over batches that mix new members (random join
    positions) and existing ones."""
    import numpy as np

    rng = np.random.default_rng(3)
    n = 5000
    names = ["10.1.%d.%d:3000" % (i >> 8, i & 255) for i in range(n)]
    a = orc.Members(names, local=names[0], join_seed=11)
    b = orc.Members(names, local=names[0], join_seed=11)
    orders = []
    for step in range(40):
        k = int(rng.integers(1, 400))
        ids = rng.integers(0, n if step > 5 else n // 4, k).astype(np.uint32)
        st = rng.integers(0, 4, k).astype(np.uint8)
        inc = rng.integers(1, 50, k).astype(np.int64)
        ra = a.update_ids(ids, st, inc, False, 1000 + step)
        rb = b.update_ids(ids, st, inc, False, 1000 + step)
        assert ra[3] == rb[3]
        orders.append(a.order())
    assert b.order() == orders[-1]
    assert len(set(orders[-1])) == len(orders[-1]) == a.count()
    # every read is a prefix-consistent snapshot: members keep their relative order as others join
    for o1, o2 in zip(orders, orders[1:]):
        pos = {x: i for i, x in enumerate(o2)}
        assert all(pos[x] < pos[y] for x, y in zip(o1, o1[1:]))
