"""Regenerate tests/golden/damp_golden.json by running the REFERENCE Membership / Member damp
scoring (lib/membership/member.js:45-66,133-153, index.js:249-324,374-383) in node here (needs
/root/reference and the oracle/_ref shims; never runs on the GPU box).

    python tests/golden/make_damp_golden.py

Inputs come from a seeded Python RNG: addresses, batches of (address, status, incarnation)
changes, clock steps, decayer ticks, the ready/set bootstrap path and per-case config values.
Outputs are data only (tests/golden/ref_damp.js): after every op, each member's dampScore,
lastUpdateDampScore and lastUpdateTimestamp, the members whose score crossed the suppress
limit (in event order), the applied change indices, and every (exponent, Math.pow(Math.E, y))
pair the engine evaluated.
"""
import json
import os
import random
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("RINGPOP_REFERENCE", "/root/reference")
STATUSES = ["alive", "suspect", "faulty", "leave"]
T0 = 1434401518824


def addr(i):
    return "10.%d.%d.%d:3000" % (i >> 16, (i >> 8) & 255, i & 255)


def random_case(name, rng, n, nops, batch, config=None, p_decay=0.3, max_step=120_000, p_same=0.1,
                with_local=True):
    members = [addr(i + 1) for i in range(n)]
    local = members[0]
    inc = {a: T0 + rng.randrange(10 ** 6) for a in members}
    now = T0 + 5_000
    ops = [{"type": "update", "now": now, "isLocal": False,
            "changes": [[a, "alive", inc[a]] for a in members]}]
    for _ in range(nops):
        if rng.random() >= p_same:
            now += rng.randrange(1, max_step)
        if rng.random() < p_decay:
            ops.append({"type": "decay", "now": now})
            continue
        ch = []
        for _ in range(rng.randrange(1, batch + 1)):
            a = rng.choice(members if with_local else members[1:])
            inc[a] += rng.choice([-1, 0, 0, 1, 1, 2])
            ch.append([a, rng.choice(STATUSES), inc[a]])
        ops.append({"type": "update", "now": now, "isLocal": rng.random() < 0.1, "changes": ch})
    return {"name": name, "local": local, "config": config or {}, "ops": ops}


def flap_case():
    """member_test.js 'flaps until exceeds suppress limit' at scale: alternating suspect / alive
    refutations one second apart, penalty 251, max 1000, suppress limit 500."""
    members = [addr(i + 1) for i in range(6)]
    ops = [{"type": "update", "now": T0, "changes": [[a, "alive", 10] for a in members]}]
    now, inc = T0, 10
    for k in range(30):
        now += 1000
        inc += 1
        st = "suspect" if k % 2 == 0 else "alive"
        ops.append({"type": "update", "now": now, "changes": [[a, st, inc] for a in members[1:]]})
        if k % 7 == 6:
            ops.append({"type": "decay", "now": now + 500})
    return {"name": "flap", "local": members[0],
            "config": {"dampScoringMax": 1000, "dampScoringSuppressLimit": 500, "dampScoringPenalty": 251},
            "ops": ops}


def half_life_case():
    """Decays at exact multiples of the half-life from odd scores: the product lands on x.5, where
    Math.round's half-up rule and the last ulp of Math.pow decide the result."""
    members = [addr(i + 1) for i in range(9)]
    ops = [{"type": "update", "now": T0, "changes": [[a, "alive", 1] for a in members]}]
    now = T0 + 1000
    # one penalty each: score = penalty (odd), lastUpdateTimestamp = now
    ops.append({"type": "update", "now": now, "changes": [[a, "suspect", 1] for a in members[1:]]})
    for k in [1, 2, 3, 4, 5, 8, 10]:
        ops.append({"type": "decay", "now": now + k * 7 * 1000})
    now2 = now + 3 * 7 * 1000
    ops.append({"type": "update", "now": now2, "changes": [[a, "faulty", 1] for a in members[1:5]]})
    for k in [1, 2, 6]:
        ops.append({"type": "decay", "now": now2 + k * 7 * 1000})
    return {"name": "half-life", "local": members[0],
            "config": {"dampScoringPenalty": 251, "dampScoringHalfLife": 7, "dampScoringMax": 100000,
                       "dampScoringSuppressLimit": 1000000}, "ops": ops}


def bootstrap_case(rng):
    """Remote changes stashed before ready, merged by set() (fresh Members, initial score), then
    updates including overrides about the local member (no self-penalty)."""
    members = [addr(i + 1) for i in range(30)]
    local = members[0]
    ops = [{"type": "ready", "value": False, "now": T0}]
    for b in range(3):
        ops.append({"type": "update", "now": T0 + b, "isLocal": False,
                    "changes": [[a, rng.choice(STATUSES[:3]), 100 + rng.randrange(5)] for a in rng.sample(members, 20)]})
    ops.append({"type": "set", "now": T0 + 10})
    ops.append({"type": "ready", "value": True, "now": T0 + 10})
    now = T0 + 10
    for _ in range(25):
        now += rng.randrange(200, 40_000)
        ch = [[a, rng.choice(STATUSES), 100 + rng.randrange(8)] for a in rng.sample(members, 8)]
        ch.append([local, rng.choice(["suspect", "faulty"]), 100 + rng.randrange(3)])
        ops.append({"type": "update", "now": now, "isLocal": rng.random() < 0.3, "changes": ch})
        if rng.random() < 0.4:
            ops.append({"type": "decay", "now": now + rng.randrange(1, 5000)})
    return {"name": "bootstrap", "local": local, "config": {"dampScoringInitial": 120}, "ops": ops}


def make_cases():
    rng = random.Random(4242)
    return [
        random_case("defaults", rng, 60, 90, 40),
        flap_case(),
        half_life_case(),
        random_case("min-floor", rng, 40, 60, 30, config={"dampScoringMin": 100, "dampScoringPenalty": 100,
                                                            "dampScoringMax": 1000, "dampScoringSuppressLimit": 700},
                    max_step=20_000),
        random_case("disabled", rng, 30, 40, 20, config={"dampScoringEnabled": False, "dampScoringInitial": 250}),
        random_case("fractional", rng, 50, 60, 25, config={"dampScoringPenalty": 333.25, "dampScoringHalfLife": 0.75,
                                                             "dampScoringInitial": 17.5, "dampScoringMin": 2.25},
                    max_step=3_000),
        bootstrap_case(rng),
        random_case("wide", rng, 1000, 24, 400, p_decay=0.25),
    ]


def main():
    cases = make_cases()
    env = dict(os.environ, NODE_PATH=os.path.join(REPO, "oracle", "_ref", "node_modules"))
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.json"), os.path.join(td, "out.json")
        with open(fin, "w") as f:
            json.dump({"cases": cases}, f)
        subprocess.check_call(["node", os.path.join(HERE, "ref_damp.js"), REF, fin, fout], env=env)
        with open(fout) as f:
            res = json.load(f)
    for c, o in zip(cases, res["cases"]):
        c["out"] = o["ops"]
    with open(os.path.join(HERE, "damp_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_damp_golden.py + ref_damp.js over lib/membership/{index,member}.js",
                   "node": res["node"], "cases": cases}, f)


if __name__ == "__main__":
    main()
