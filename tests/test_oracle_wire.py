"""The wire-body oracle (oracle/pywire.py) against the reference's own output
(tests/golden/wire_golden.json: lib/gossip/dissemination.js run in node by
tests/golden/make_wire_golden.py). CPU only."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import pywire  # noqa: E402


def golden():
    with open(os.path.join(HERE, "golden", "wire_golden.json")) as f:
        return json.load(f)["cases"]


def test_oracle_matches_reference_wire_text():
    for c in golden():
        recs = [pywire.issue_as_record(ch[5], ch[3], ch[4], ch[0], ch[1], ch[2]) for ch in c["changes"]]
        fs = [pywire.full_sync_record(c["whoami"], m[0], m[1], m[2]) for m in c["members"]]
        o = c["out"]
        assert pywire.body(recs) == o["issueAs"], c["name"]
        assert pywire.body(fs) == o["fullSync"], c["name"]
        assert pywire.body(recs, "ping", c["checksum"], c["whoami"], c["whoamiInc"]) == o["ping"], c["name"]
        assert pywire.body(recs, "pingResponse") == o["pingResponse"], c["name"]
        assert pywire.decode(o["ping"]) == recs
        assert pywire.body(recs, "pingReq", c["checksum"], c["whoami"], c["whoamiInc"],
                           target=c["target"]) == o["pingReq"], c["name"]
        assert pywire.body(recs, "pingReqResponse", target=c["target"], ping_status=c["pingStatus"]) == \
            o["pingReqResponse"], c["name"]
        assert pywire.body(fs, "joinResponse", c["checksum"], c["whoami"], app=c["app"]) == o["joinResponse"], c["name"]
        assert pywire.decode(o["joinResponse"]) == fs


def _all_texts():
    import wire_texts as wt
    cases = wt.golden()
    names = set(wt.golden_names(cases))
    texts = [t for seed in range(11, 21) for t in wt.fuzz_texts(cases, seed)]
    for make in (wt.long_array_texts, wt.many_member_texts, wt.big_byte_texts):
        n, t = make()
        names |= set(n)
        texts += t
    names = sorted(names)
    ids = {n.encode(): i for i, n in enumerate(names)}
    return texts, ids


def test_decoder_contract_pinned_by_json_loads():
    """oracle/pywire.decode_columns (the decoder's contract) against Python's json.loads on every
    wire-decoder test text: a JSON-valid text is accepted exactly when json.loads finds it within
    the contract, and then every record column and header equals json.loads's reading of it. The
    JSON-invalid mutants are rejected except where the contract's lenient skip of unknown members
    or its leading-zero integers let them through (counted)."""
    import wire_texts as wt
    texts, ids = _all_texts()
    n_valid = n_ok = lenient = 0
    for t in texts:
        b = t.encode()
        got = pywire.decode_columns(b, ids)
        want = wt.json_contract(t, ids)
        if want is None:
            lenient += got["err"] == 0
            continue
        n_valid += 1
        assert (got["err"] == 0) == want["ok"], t[:300]
        if not want["ok"]:
            continue
        n_ok += 1
        assert len(got["records"]) == len(want["records"]), t[:300]
        for g, w in zip(got["records"], want["records"]):
            assert (g["addr"], g["src"], g["status"], g["inc"], g["src_inc"]) == \
                (w["addr"], w["src"], w["status"], w["inc"], w["src_inc"])
            assert b[g["addr_off"]:g["addr_off"] + g["addr_len"]].decode() == w["addr_name"]
            if w["id"] is None:
                assert g["id_off"] is None
            else:
                assert b[g["id_off"]:g["id_off"] + len(w["id"].encode())].decode() == w["id"]
                assert b[g["id_off"] + len(w["id"].encode())] == ord('"')
        for col in ("checksum", "source", "source_inc", "target", "ping_status"):
            assert got[col] == want[col], (col, t[:300])
    assert n_valid > 2000 and n_ok > 1800 and len(texts) - n_valid > 400, (n_valid, n_ok, len(texts))
    assert lenient < 0.2 * (len(texts) - n_valid), lenient


def test_decoder_contract_rejections():
    """The contract's rejections (escapes, fractions / exponents, 19-digit numbers, a bad status,
    a missing member, trailing bytes, truncation) and their byte offsets (err = 1 + offset)."""
    ids = {b"10.0.0.1:1": 0}
    ok = '[{"address":"10.0.0.1:1","status":"alive","incarnationNumber":%s}]'
    assert pywire.decode_columns(ok % "7", ids)["err"] == 0
    assert pywire.decode_columns(ok % "1.5", ids)["err"] == 1 + (ok % "1.5").index("1.5") + 1
    assert pywire.decode_columns(ok % "1e5", ids)["err"] == 1 + (ok % "1e5").index("e5")
    assert pywire.decode_columns(ok % ("1" * 19), ids)["err"] == 1 + (ok % "1").index("1}") + 19
    assert pywire.decode_columns(ok % ("9" * 18), ids)["records"][0]["inc"] == 10 ** 18 - 1
    esc = '[{"address":"10.0\\u002e0.1:1","status":"alive","incarnationNumber":1}]'
    assert pywire.decode_columns(esc, ids)["err"] == 1 + esc.index("\\")
    miss = '[{"address":"10.0.0.1:1","status":"alive"}]'
    assert pywire.decode_columns(miss, ids)["err"] == 1 + miss.index("}") + 1
    dead = '[{"address":"10.0.0.1:1","status":"dead","incarnationNumber":1}]'
    assert pywire.decode_columns(dead, ids)["err"] > 0
    assert pywire.decode_columns((ok % "7") + " x", ids)["err"] == 1 + len(ok % "7") + 1
    assert pywire.decode_columns((ok % "7")[:-1], ids)["err"] == 1 + len(ok % "7") - 1
    assert pywire.decode_columns('{"checksum":1}', ids)["err"] == 1 + len('{"checksum":1}')
    assert pywire.decode_columns("", ids)["err"] == 1
    skip = '{"x":[1,{"b":"]"}],"changes":[],"y":3.5e2,"checksum":-1}'
    got = pywire.decode_columns(skip, ids)
    assert got["err"] == 0 and got["checksum"] == 0xFFFFFFFF and got["records"] == []
