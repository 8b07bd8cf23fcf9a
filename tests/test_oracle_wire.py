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
