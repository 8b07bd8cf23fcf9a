"""Time the REFERENCE JavaScript on this host (tools/ref_node_bench.js) at C1, C2 and C3 and
print the results as JSON (recorded in BASELINE.md §3). Needs /root/reference and node; the
reference's farmhash dependency is served by the oracle's N-API module (make -C oracle ref).

    python tools/ref_node_bench.py > profiles/r02/ref_node_bench.json
"""
import json
import os
import platform
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("RINGPOP_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import pyoracle  # noqa: E402
from sim_configs import synth  # noqa: E402


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all", "ref"])
    S = synth()
    with open(os.path.join(REF, "benchmarks", "large-membership.json")) as f:
        large = [m["address"] for m in json.load(f)]
    keys = [k.tobytes().decode() for k in pyoracle.uuid_keys(42, 0, 1_000_000)]
    rings = [
        {"name": "C1", "servers": large[:1000], "keys": keys, "lookupNKeys": 100_000},
        {"name": "C2", "servers": [S.c2_addr(i) for i in range(10_000)], "keys": keys, "lookupNKeys": 10_000,
         "extra": [S.c2_addr(11_000 + i) for i in range(20)]},
    ]
    n = k = 100_000
    names, _, inc0 = S.c3_members(n)
    batches = []
    for b in range(5):
        ids, us, ui = S.c3_updates(n, k, seed=100 + b, base_inc=inc0 + 3 * b)
        batches.append({"ids": ids.tolist(), "st": us.tolist(), "inc": [int(x) for x in ui]})
    mems = [{"name": "C3", "names": names, "inc0": [int(x) for x in inc0], "batches": batches}]
    env = dict(os.environ, NODE_PATH=os.path.join(REPO, "oracle", "_ref", "node_modules"))
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.json"), os.path.join(td, "out.json")
        with open(fin, "w") as f:
            json.dump({"rings": rings, "memberships": mems}, f)
        subprocess.check_call(["node", "--max-old-space-size=8192", os.path.join(REPO, "tools", "ref_node_bench.js"),
                               REF, fin, fout], env=env)
        with open(fout) as f:
            res = json.load(f)
    model = None
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    res["host"] = {"cpu_model": model, "nproc": os.cpu_count(), "threads_used": 1, "python": platform.python_version()}
    res["note"] = ("reference lib/ring + lib/membership JS, single thread (Node event loop), farmhash = the oracle's "
                   "N-API restatement; C1 = benchmarks/large-membership.json[0:1000] servers, C2 = 10k C2 addresses, "
                   "keys = 1M Philox UUIDs (seed 42); C3 = 100k members, 5 fresh batches of 100k updates")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
