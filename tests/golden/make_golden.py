"""Regenerate the committed golden fixtures under tests/golden/ by running the REFERENCE
JavaScript in this container (needs /root/reference and node; never runs on the GPU box).

    python tests/golden/make_golden.py [ring]

Inputs are built with the oracle's Philox / uuid stream (oracle/pyoracle.py); the reference's
`farmhash` dependency is served by the oracle's N-API restatement (oracle/gen/farmhash_napi.c),
built into oracle/_ref/ by `make -C oracle ref`. Outputs are data only: inputs + what the
reference returned.
"""
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("RINGPOP_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle  # noqa: E402


def run_node(script, cases):
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all", "ref"])
    env = dict(os.environ, NODE_PATH=os.path.join(REPO, "oracle", "_ref", "node_modules"))
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.json"), os.path.join(td, "out.json")
        with open(fin, "w") as f:
            json.dump({"cases": cases}, f)
        subprocess.check_call(["node", os.path.join(HERE, script), REF, fin, fout], env=env)
        with open(fout) as f:
            return json.load(f)["cases"]


def tree_digest(tree):
    h = hashlib.sha256()
    for t, o in zip(tree["tokens"], tree["owners"]):
        h.update(("%d:%s;" % (t, o)).encode())
    return h.hexdigest()


def ring_cases():
    with open(os.path.join(REF, "benchmarks", "large-membership.json")) as f:
        large = [m["address"] for m in json.load(f)]
    servers = large[:1000]
    extra = large[1000:1005]
    keys = [k.tobytes().decode() for k in pyoracle.uuid_keys(42, 0, 4096)]
    uk = lambda seed, k0, n: {"uuid": [seed, k0, n]}  # noqa: E731
    rng = random.Random(1234)

    cases = []
    # C1: benchmarks/add-remove-hashring.js servers, real farmhash, 1000 x 100 points
    removed = servers[::10]
    cases.append({
        "name": "c1", "hashKind": "farmhash", "dump": True,
        "batches": [
            dict({"add": servers, "remove": [], "keys": keys, "ns": [1, 3]}, uuid=uk(42, 0, 4096)),
            dict({"add": extra, "remove": removed, "keys": keys[:1024], "ns": [3]}, uuid=uk(42, 0, 1024)),
            dict({"add": [], "remove": ["10.99.99.99:1"], "keys": keys[:16], "ns": [3]}, uuid=uk(42, 0, 16)),
        ],
    })
    # Forced collisions: farmhash % 2000 through the hashFunc injection point, 120 servers
    # x 20 points, random add/remove histories with duplicates and add+remove in one batch.
    pool = ["10.1.%d.%d:%d" % (i // 50, i % 50, 3000 + i) for i in range(120)]
    batches = []
    for b in range(16):
        add = rng.sample(pool, rng.randint(0, 40))
        add += rng.sample(add, min(len(add), rng.randint(0, 3)))  # duplicates in one batch
        rem = rng.sample(pool, rng.randint(0, 30))
        if add and rng.random() < 0.5:
            rem.append(add[0])  # added then removed in the same batch
        probes = sorted(set([0, 1, 1999, 2000, 4294967295] + [rng.randrange(0, 2100) for _ in range(60)]))
        batches.append({"add": add, "remove": rem, "keys": ["#%d" % p for p in probes],
                        "ns": [-1, 0, 1, 2, 3, 7, 200]})
    batches.append({"add": [], "remove": pool, "keys": ["#0", "#5"], "ns": [0, 1, 3]})
    batches.append({"add": pool[:2], "remove": [], "keys": ["#0", "#1999", "#2001"], "ns": [-1, 0, 1, 2, 3, 5]})
    cases.append({"name": "collide", "hashKind": "mod", "hashMod": 2000, "replicaPoints": 20,
                  "dump": True, "batches": batches})
    # test/unit/ring-test.js:82-124 known answers (extractPort hashFunc)
    ports = ["127.0.0.1:%d" % (3000 + i) for i in range(1000)]
    cases.append({"name": "port", "hashKind": "port", "dump": True, "batches": [
        {"add": ports, "remove": [], "keys": [p + "0" for p in ports], "ns": [3]},
    ]})
    cases.append({"name": "port1", "hashKind": "port", "dump": True, "batches": [
        {"add": [], "remove": [], "keys": [ports[0] + "0"], "ns": [3]},
        {"add": [ports[0]], "remove": [], "keys": [ports[0] + "0", "127.0.0.1:99999"], "ns": [-2, 0, 1, 3]},
    ]})
    # tiny farmhash rings: wrap-around, n > servers, n <= 0
    tiny_keys = [k.tobytes().decode() for k in pyoracle.uuid_keys(7, 0, 64)]
    cases.append({"name": "tiny", "hashKind": "farmhash", "replicaPoints": 3, "dump": True, "batches": [
        dict({"add": ["a"], "remove": [], "keys": tiny_keys, "ns": [-1, 0, 1, 2, 5]}, uuid=uk(7, 0, 64)),
        dict({"add": ["b", "test 1", "a"], "remove": [], "keys": tiny_keys, "ns": [-1, 0, 1, 2, 3, 5]},
             uuid=uk(7, 0, 64)),
        dict({"add": [], "remove": ["a"], "keys": tiny_keys, "ns": [1, 2, 3]}, uuid=uk(7, 0, 64)),
    ]})
    return cases


def make_ring():
    cases = ring_cases()
    outs = run_node("ref_ring.js", cases)
    fixture = {"generator": "tests/golden/make_golden.py + tests/golden/ref_ring.js",
               "reference": "lib/ring/index.js, lib/ring/rbtree.js (ringpop v10.9.6)",
               "note": "owners are indices into the case's `names` (-1 = null); uuid keys are "
                       "[seed, k0, n] of the oracle's Philox uuid stream",
               "cases": []}
    for c, o in zip(cases, outs):
        names, index = [], {}

        def nid(s):
            if s is None:
                return -1
            if s not in index:
                index[s] = len(names)
                names.append(s)
            return index[s]

        fc = {"name": c["name"], "hashKind": c["hashKind"], "hashMod": c.get("hashMod"),
              "replicaPoints": c.get("replicaPoints", 100), "names": names, "batches": []}
        for b, ob in zip(c["batches"], o["batches"]):
            fb = {"add": b["add"], "remove": b["remove"], "changed": ob["changed"],
                  "checksum": ob["checksum"], "serverCount": ob["serverCount"], "size": ob["size"],
                  "servers": ob["servers"]}  # Object.keys(ring.servers): insertion order
            tree = ob["tree"]
            fb["tree_sha256"] = tree_digest(tree)
            if len(tree["tokens"]) <= 4000:
                fb["tree"] = {"tokens": tree["tokens"], "owners": [nid(x) for x in tree["owners"]]}
            if "keys" in b:
                fb["keys"] = b.get("uuid") or b["keys"]
                fb["lookup"] = [nid(x) for x in ob["lookup"]]
                fb["lookupN"] = {n: [[nid(x) for x in lst] for lst in v] for n, v in ob["lookupN"].items()}
            fc["batches"].append(fb)
        fixture["cases"].append(fc)
    path = os.path.join(HERE, "ring_golden.json")
    with open(path, "w") as f:
        json.dump(fixture, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


JOIN_TAG = 0x4A4F494E  # 'JOIN' — key[1] of the getJoinPosition Philox stream (oracle/orc_members.c)


def join_rands(seed, n):
    return [pyoracle.philox([k, 0, 0, 0], [seed, JOIN_TAG])[0] for k in range(n)]


def membership_cases():
    with open(os.path.join(REF, "benchmarks", "large-membership.json")) as f:
        large = json.load(f)
    addrs = [m["address"] for m in large]
    statuses = ["alive", "suspect", "faulty", "leave"]
    cases = []
    # 1. the override table (member.js:71-202) for a remote and the local member
    local = "127.0.0.1:3000"
    for tgt in ("remote", "local"):
        addr = local if tgt == "local" else "127.0.0.1:3001"
        for cur in statuses:
            for upd in statuses:
                for d in (-1, 0, 1):
                    ops = []
                    if tgt == "remote":
                        ops.append({"type": "update", "changes": [[local, "alive", 1]], "isLocal": True, "now": 1})
                    ops.append({"type": "update", "changes": [[addr, cur, 100]], "now": 2})
                    ops.append({"type": "update", "changes": [[addr, upd, 100 + d]], "now": 777, "members": True})
                    cases.append({"name": "rule/%s/%s/%s/%+d" % (tgt, cur, upd, d), "local": local,
                                  "joinSeed": 1, "joinRands": join_rands(1, 4), "ops": ops})
    # 2. random batches with duplicate addresses, new members and local updates
    rng = random.Random(77)
    names = addrs[:300]
    local = names[0]
    incs = {a: 1434401518824 + rng.randrange(10 ** 6) for a in names}
    ops = [{"type": "update", "changes": [[local, "alive", incs[local]]], "isLocal": True, "now": 5},
           {"type": "update", "changes": [[a, "alive", incs[a]] for a in names[1:]], "now": 6, "members": True,
            "checksumString": True}]
    pool = list(names)
    for b in range(8):
        changes = []
        for _ in range(600):
            r = rng.random()
            if r < 0.03:
                a = addrs[300 + rng.randrange(100)]
            elif r < 0.08:
                a = local
            elif r < 0.38 and changes:
                a = changes[rng.randrange(len(changes))][0]  # duplicate address in one batch
            else:
                a = rng.choice(pool)
            st = rng.choices(statuses, weights=[50, 25, 15, 10])[0]
            base = incs.get(a, 1434401518824)
            inc = base + rng.choice([-1, 0, 0, 1, 1, 2, 1000])
            changes.append([a, st, inc])
        ops.append({"type": "update", "changes": changes, "now": 1434500000000 + b, "members": True,
                    "checksumString": b == 7})
    cases.append({"name": "random", "local": local, "joinSeed": 2, "joinRands": join_rands(2, 2000), "ops": ops})
    # 3. the 1332-member fixture (benchmarks/large-membership.json) then a mixed batch
    local = addrs[0]
    ops = [{"type": "update", "changes": [[local, "alive", large[0]["incarnationNumber"]]], "isLocal": True,
            "now": 7},
           {"type": "update", "changes": [[m["address"], m["status"], m["incarnationNumber"]] for m in large[1:]],
            "now": 8, "checksumString": True}]
    changes = []
    for _ in range(2000):
        m = rng.choice(large)
        changes.append([m["address"], rng.choice(statuses), m["incarnationNumber"] + rng.choice([-1, 0, 1])])
    ops.append({"type": "update", "changes": changes, "now": 9, "members": True})
    cases.append({"name": "fixture1332", "local": local, "joinSeed": 3, "joinRands": join_rands(3, 4000), "ops": ops})
    # 4. stash until ready, then set() (index.js:208-265, merge.js:22-51)
    local = "127.0.0.1:3000"
    peers = ["127.0.0.1:%d" % (3001 + i) for i in range(6)]
    ops = [{"type": "ready", "value": False},
           {"type": "update", "changes": [[local, "alive", 10]], "isLocal": True, "now": 1},
           {"type": "update", "changes": [[peers[0], "suspect", 1], [peers[1], "alive", 2], [local, "faulty", 99]]},
           {"type": "update", "changes": [[peers[0], "alive", 2], [peers[1], "suspect", 1], [peers[2], "faulty", 1]]},
           {"type": "update", "changes": [[peers[3], "leave", 4], [peers[0], "faulty", 2], [peers[4], "alive", 9]]},
           {"type": "set", "members": True},
           {"type": "ready", "value": True},
           {"type": "update", "changes": [[peers[5], "alive", 1], [peers[2], "alive", 5]], "members": True}]
    cases.append({"name": "stash-set", "local": local, "joinSeed": 4, "joinRands": join_rands(4, 10), "ops": ops})
    # 5. membership_test.js:58-146 style: leave overrides and redundant leaves
    a = "127.0.0.1:3001"
    ops = [{"type": "update", "changes": [[local, "alive", 50]], "isLocal": True, "now": 1},
           {"type": "update", "changes": [[a, "alive", 100]]},
           {"type": "update", "changes": [[a, "leave", 100]]},
           {"type": "update", "changes": [[a, "leave", 100]]},
           {"type": "update", "changes": [[local, "leave", 50]]},
           {"type": "update", "changes": [[local, "leave", 51]], "members": True},
           {"type": "update", "changes": [[local, "suspect", 51], [a, "alive", 101], [a, "leave", 101]],
            "now": 4242, "members": True}]
    cases.append({"name": "leave", "local": local, "joinSeed": 5, "joinRands": join_rands(5, 10), "ops": ops})
    return cases


def make_membership():
    cases = membership_cases()
    outs = run_node("ref_membership.js", cases)
    fixture = {"generator": "tests/golden/make_golden.py + tests/golden/ref_membership.js",
               "reference": "lib/membership/index.js, member.js, merge.js (ringpop v10.9.6)",
               "note": "changes are [address, status, incarnationNumber]; applied = [change index, status, inc] "
                       "in return order; joinRands feed getJoinPosition (floor(r/2^32*len))",
               "cases": []}
    for c, o in zip(cases, outs):
        fops = []
        for op, oo in zip(c["ops"], o["ops"]):
            f = dict(op)
            f.update(oo)
            fops.append(f)
        fixture["cases"].append({"name": c["name"], "local": c["local"], "joinSeed": c["joinSeed"], "ops": fops})
    path = os.path.join(HERE, "membership_golden.json")
    with open(path, "w") as f:
        json.dump(fixture, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


def synth():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def sim_cases():
    S = synth()
    cases = []
    for name, n, k, rounds, susp, seed in [("n16k1", 16, 1, 40, 25, 11), ("n64k2", 64, 2, 45, 25, 11),
                                           ("n128k3-susp4", 128, 3, 30, 4, 5), ("n200k10", 200, 10, 50, 25, 11)]:
        cases.append({"name": name, "names": [S.c2_addr(i) for i in range(n)],
                      "inc0": [int(x) for x in S.c3_members(n)[2]],
                      "dead": [int(x) for x in S.kill_set(n, k, seed)], "seed": seed, "suspRounds": susp,
                      "now0": S.NOW0, "rounds": rounds, "views": [0, n - 1]})
    # Scenario cases: the branches the kill-only cases never take.
    #  - n100k1-digits: the ring server count crosses a power of ten (100 -> 99), so
    #    adjustMaxPiggybackCount (dissemination.js:38-55) re-values maxPiggybackCount 45 -> 30
    #  - n40-leave: admin leave (server/admin/member.js:92-93 -> makeLeave) as the convergence
    #    scenarios send it, plus a node that crashes mid-run (it had started gossiping)
    #  - n64-half-leave: benchmarks/convergence-time/scenarios/half-cluster-failure.js (half the
    #    hosts leave at once)
    #  - n24-revive: a node down from round 0 comes back after every change about it expired:
    #    it is answered with a full sync (dissemination.js:100-114) and refutes its own faulty
    #    status (member.js:76-81); a second node is suspended briefly and refutes `suspect`
    #  - n30-join / n70-join: fresh processes bootstrapping into the running cluster from join
    #    responses (mergeJoinResponses -> set(), join-sender.js:253-256): crashed nodes come back
    #    after they were declared faulty, a live node restarts, a node that left rejoins, and
    #    several nodes join in one round (later joiners may be answered by earlier ones)
    ev = lambda *e: [list(x) for x in e]  # noqa: E731
    scen = [("n100k1-digits", 100, 1, 60, 25, 13, []),
            ("n40-leave", 40, 1, 70, 6, 17, ev((2, "leave", 3), (5, "kill", 9), (10, "leave", 7), (11, "leave", 7),
                                              (30, "leave", 20), (30, "kill", 21))),
            ("n64-half-leave", 64, 0, 60, 25, 19, ev(*[(1, "leave", v) for v in range(0, 64, 2)])),
            ("n24-revive", 24, 0, 110, 8, 23, ev((0, "kill", 4), (3, "kill", 6), (12, "revive", 6),
                                                 (60, "revive", 4), (70, "kill", 11), (71, "leave", 12))),
            ("n30-join", 30, 0, 95, 6, 29, ev((0, "kill", 4), (0, "kill", 9), (5, "leave", 8), (22, "join", 4),
                                               (28, "join", 13), (30, "join", 8), (45, "join", 9), (46, "kill", 2))),
            ("n70-join", 70, 0, 80, 7, 31, ev(*([(3, "kill", v) for v in range(10, 16)] +
                                                [(33, "join", v) for v in range(10, 16)])))]
    for name, n, k, rounds, susp, seed, events in scen:
        cases.append({"name": name, "names": [S.c2_addr(i) for i in range(n)],
                      "inc0": [int(x) for x in S.c3_members(n)[2]],
                      "dead": [int(x) for x in S.kill_set(n, k, seed)] if k else [0] * n, "seed": seed,
                      "suspRounds": susp, "now0": S.NOW0, "rounds": rounds,
                      "views": [0, n - 1] + sorted({e[2] for e in events if e[1] == "join"})[:2],
                      "events": events})
    return cases


def make_sim():
    cases = sim_cases()
    outs = run_node("ref_sim.js", cases)
    fixture = {"generator": "tests/golden/make_golden.py + tests/golden/ref_sim.js",
               "reference": "lib/membership/*, lib/gossip/{dissemination,suspicion}.js, lib/membership/iterator.js, "
                            "lib/ring, lib/on_membership_event.js (ringpop v10.9.6) in the round model of "
                            "oracle/orc_sim.c",
               "note": "checksums[r][v] = node v's membership checksum after round r (0 while v is down); "
                       "maxPiggyback[r][v] = v's dissemination.maxPiggybackCount after round r; fullSyncs = "
                       "full syncs the reference sent (its 'full-sync' stat); events [round, kind, node] run "
                       "before that round; finalViews = members arrays [address, status, inc] of the listed "
                       "nodes",
               "cases": []}
    for c, o in zip(cases, outs):
        f = {k: c[k] for k in ("name", "seed", "suspRounds", "now0", "rounds", "views")}
        f["n"] = len(c["names"])
        f["dead"] = c["dead"]
        f["events"] = c.get("events", [])
        f["checksums"] = o["rounds"]
        f["maxPiggyback"] = o["maxPiggyback"]
        f["fullSyncs"] = o["fullSyncs"]
        f["finalViews"] = o["finalViews"]
        fixture["cases"].append(f)
    path = os.path.join(HERE, "sim_golden.json")
    with open(path, "w") as fh:
        json.dump(fixture, fh, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    what = sys.argv[1:] or ["ring", "membership", "sim"]
    if "ring" in what:
        make_ring()
    if "membership" in what:
        make_membership()
    if "sim" in what:
        make_sim()
