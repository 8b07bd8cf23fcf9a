"""GPU parity of the Node N-API host (ringpop-node_amd/js): the reference's JS API
(HashRing, GossipSim) driven from node against the reference goldens. Each test runs one
node process (tests/js/*.js) that reports its mismatches as JSON."""
import json
import os
import shutil
import subprocess

import pytest

import golden_util as gu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(shutil.which("node") is None, reason="node not in this image")]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_node(script, payload, tmp_path):
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "ringpop-node_amd", "js")])
    inp = tmp_path / "in.json"
    inp.write_text(json.dumps(payload))
    out = subprocess.run(["node", os.path.join(REPO, "tests", "js", script), str(inp)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_js_hashring_matches_reference_goldens(gpu, tmp_path):
    cases = gu.load("ring_golden.json")["cases"]
    for c in cases:
        for b in c["batches"]:
            if "keys" in b:
                b["keys"] = gu.keys_of(b)
            b.pop("tree", None)
    res = run_node("ring_parity.js", {"cases": cases}, tmp_path)
    assert res["nfail"] == 0, res["fails"]
    assert res["checks"] > 400


def test_js_hashring_inherited_names_match_reference(gpu, tmp_path):
    """Single add / remove / addRemoveServers / hasServer calls with names the servers map
    inherits from Object.prototype ('constructor', 'toString', ...) and ordinary names, against
    the reference's own results (tests/golden/make_ring_ops.py): a removal of an inherited name
    reports a change, recomputes the checksum and emits 'removed' without touching the device."""
    res = run_node("ring_ops_parity.js", {"cases": gu.load("ring_ops_golden.json")["cases"]}, tmp_path)
    assert res["nfail"] == 0, res["fails"]
    assert res["checks"] >= 70


def test_js_gossipsim_matches_reference_goldens(gpu, tmp_path):
    import importlib.util
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    S = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(S)
    cases = []
    golden = gu.load("sim_golden.json")["cases"]
    for c in golden[:2] + [x for x in golden if x["name"] in ("n24-revive", "n30-join")]:
        n = c["n"]
        cases.append(dict(c, names=[S.c2_addr(i) for i in range(n)], inc0=[int(x) for x in S.c3_members(n)[2]]))
    res = run_node("sim_parity.js", {"cases": cases}, tmp_path)
    assert res["nfail"] == 0, res["fails"]


def test_js_membership_dropin_matches_reference_goldens(gpu, tmp_path):
    """The drop-in lib/membership module (ringpop-node_amd/js/membership.js), installed into the
    module cache the way a ringpop deployment installs it, replays every membership golden: the
    96 override rules (remote + local), random batches with repeated addresses and local
    overrides, the 1332-member fixture, stash + set(), and the leave cases; then every damp
    scoring golden (tests/golden/damp_golden.json) with the scores on the device."""
    import pyoracle
    cases = gu.load("membership_golden.json")["cases"]
    for c in cases:
        n = 4000 if c["name"] == "fixture1332" else 2000
        c["joinRands"] = [pyoracle.philox([k, 0, 0, 0], [c["joinSeed"], 0x4A4F494E])[0] for k in range(n)]
    damp = gu.load("damp_golden.json")["cases"]
    for c in damp:
        for o in c["out"]:
            o.pop("pow", None)
    res = run_node("membership_parity.js", {"cases": cases, "dampCases": damp}, tmp_path)
    assert res["nfail"] == 0, res["fails"]
    assert res["checks"] > 700 + 2 * sum(len(c["ops"]) for c in damp)


def test_js_wire_bodies_match_reference_goldens(gpu, tmp_path):
    """rpamd.node wireEncode / wireDecode (-> rp_wire_encode / rp_wire_decode): every golden body
    — issueAs / fullSync arrays, ping, ping response, ping-req request, join response, with
    per-record undefined members — byte for byte, and the bodies decoded back."""
    res = run_node("wire_parity.js", {"cases": gu.load("wire_golden.json")["cases"]}, tmp_path)
    assert res["nfail"] == 0, res["fails"]
    assert res["checks"] > 100
