"""Regenerate tests/golden/wire_golden.json by running the REFERENCE Dissemination
(lib/gossip/dissemination.js) in node here (needs /root/reference; never runs on the GPU box).

    python tests/golden/make_wire_golden.py

Inputs: addresses from the reference's benchmarks/large-membership.json, statuses / incarnation
numbers / uuid ids from a seeded Python RNG. Outputs are data only: the inputs and the JSON text
the reference produced (tests/golden/ref_wire.js).
"""
import json
import os
import random
import subprocess
import tempfile
import uuid

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("RINGPOP_REFERENCE", "/root/reference")
STATUSES = ["alive", "suspect", "faulty", "leave"]


def make_cases():
    with open(os.path.join(REF, "benchmarks", "large-membership.json")) as f:
        large = [m["address"] for m in json.load(f)]
    rng = random.Random(77)
    cases = []
    for name, n_members, n_changes, with_ids in [("empty", 3, 0, True), ("one", 4, 1, True), ("small", 40, 25, True),
                                                 ("noid", 40, 30, False), ("wide", 600, 400, True),
                                                 ("absent", 60, 45, "mixed")]:
        members = large[:n_members]
        whoami = members[0]
        incs = [0, 1, 1434401518824, 2 ** 53 - 1, 9, 10, 99, 100]
        mem = [[a, rng.choice(STATUSES), rng.choice(incs) if rng.random() < 0.3 else 1434401518824 + rng.randrange(10 ** 6)]
               for a in members]
        changes = []
        for a in rng.sample(members, n_changes):
            src = rng.choice(members)
            ch = [a, rng.choice(STATUSES), rng.choice([rng.choice(incs), 1434401500000 + rng.randrange(10 ** 7)]),
                  src, 1434401500000 + rng.randrange(10 ** 7),
                  str(uuid.UUID(int=rng.getrandbits(128), version=4)) if with_ids else None]
            if with_ids == "mixed":  # JSON.stringify leaves undefined members out, per record
                ch[3] = None if rng.random() < 0.3 else ch[3]
                ch[4] = None if rng.random() < 0.3 else ch[4]
                ch[5] = None if rng.random() < 0.4 else ch[5]
            changes.append(ch)
        cases.append({"name": name, "whoami": whoami, "whoamiInc": 1434401518824 + rng.randrange(1000),
                      "serverCount": n_members, "checksum": rng.getrandbits(32), "members": mem, "changes": changes,
                      "target": members[-1], "pingStatus": rng.random() < 0.5, "app": "ringpop-" + name})
    return cases


def main():
    cases = make_cases()
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.json"), os.path.join(td, "out.json")
        with open(fin, "w") as f:
            json.dump({"cases": cases}, f)
        subprocess.check_call(["node", os.path.join(HERE, "ref_wire.js"), REF, fin, fout])
        with open(fout) as f:
            outs = json.load(f)["cases"]
    for c, o in zip(cases, outs):
        c["out"] = o
    with open(os.path.join(HERE, "wire_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_wire_golden.py + ref_wire.js over lib/gossip/dissemination.js",
                   "cases": cases}, f)


if __name__ == "__main__":
    main()
