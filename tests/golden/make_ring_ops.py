"""Golden vectors of single HashRing calls from the REFERENCE (lib/ring/index.js), including names
that the servers map inherits from Object.prototype ('constructor', 'toString', ...): the
reference's hasServer(name) is `!!this.servers[name]`, so such a name counts as present, an add of
it does nothing, and a remove of it removes no token yet recomputes the checksum, emits
'removed' and reports a change. Writes tests/golden/ring_ops_golden.json.

    python tests/golden/make_ring_ops.py   (needs /root/reference and node; not run on the GPU box)
"""
import json
import os

from make_golden import HERE, run_node

A = ["10.0.0.%d:3000" % i for i in range(6)]
CASES = [
    {"name": "inherited-names", "replicaPoints": 10, "ops": [
        ["addRemoveServers", A[:4], []],
        ["hasServer", "constructor"],
        ["addServer", "constructor"],
        ["removeServer", "constructor"],
        ["addRemoveServers", ["toString"], []],
        ["addRemoveServers", [], ["toString"]],
        ["addRemoveServers", [A[4]], ["valueOf", A[0]]],
        ["addRemoveServers", [], ["hasOwnProperty", "not-there"]],
        ["removeServer", "not-there"],
        ["addServer", A[5]],
        ["removeServer", A[5]],
        ["addRemoveServers", ["constructor", A[5]], ["isPrototypeOf"]],
        ["hasServer", "toString"],
        ["addRemoveServers", ["10.0.0.9:3000"], ["10.0.0.9:3000", "constructor"]],
        ["addRemoveServers", ["10.0.0.8:3000", "10.0.0.8:3000"], ["toString", "10.0.0.8:3000", A[1]]],
    ]},
]


def main():
    outs = run_node("ref_ring_ops.js", CASES)
    fixture = {"generator": "tests/golden/make_ring_ops.py + tests/golden/ref_ring_ops.js",
               "reference": "lib/ring/index.js (ringpop v10.9.6)",
               "cases": [dict(c, results=o["ops"]) for c, o in zip(CASES, outs)]}
    with open(os.path.join(HERE, "ring_ops_golden.json"), "w") as f:
        json.dump(fixture, f, indent=1)


if __name__ == "__main__":
    main()
