"""CPU restatement of the gossip wire bodies — TEST INFRASTRUCTURE ONLY (the checker of
rp_wire_*; only tests/ may import it). Pinned by tests/golden/wire_golden.json, which the
reference's own Dissemination produced (tests/golden/make_wire_golden.py).

JSON.stringify of the reference's object literals equals json.dumps with compact separators
and insertion-ordered keys for these inputs (ASCII strings without escapes, integral Numbers).
"""
import json

STATUS_NAME = ["alive", "suspect", "faulty", "leave"]


def _dumps(o):
    return json.dumps(o, separators=(",", ":"))


def issue_as_record(id_, source, source_inc, address, status, inc):
    """dissemination.js:163-170 (an undefined member is dropped, as JSON.stringify does)."""
    r = {"id": id_} if id_ is not None else {}
    if source is not None:
        r["source"] = source
    if source_inc is not None:
        r["sourceIncarnationNumber"] = source_inc
    r.update(address=address, status=status, incarnationNumber=inc)
    return r


def full_sync_record(source, address, status, inc):
    """dissemination.js:64-73."""
    return {"source": source, "address": address, "status": status, "incarnationNumber": inc}


def body(changes, kind="array", checksum=None, source=None, source_inc=None, target=None, ping_status=None,
         app=None):
    if kind == "ping":  # ping-sender.js:71-76
        return _dumps({"checksum": checksum, "changes": changes, "source": source,
                       "sourceIncarnationNumber": source_inc})
    if kind == "pingResponse":  # server/protocol/ping.js:45-48
        return _dumps({"changes": changes})
    if kind == "pingReq":  # ping-req-sender.js:75-81
        return _dumps({"checksum": checksum, "changes": changes, "source": source,
                       "sourceIncarnationNumber": source_inc, "target": target})
    if kind == "pingReqResponse":  # server/protocol/ping-req.js:61-65
        return _dumps({"changes": changes, "pingStatus": bool(ping_status), "target": target})
    if kind == "joinResponse":  # server/protocol/join.js:128-133 (membership = fullSync records)
        return _dumps({"app": app, "coordinator": source, "membership": changes, "membershipChecksum": checksum})
    return _dumps(changes)


def decode(text):
    """The changes of a body or a bare array (server/protocol/ping.js:27-36 reads `changes`; a
    join response carries them as `membership`)."""
    o = json.loads(text)
    if isinstance(o, list):
        return o
    return o["membership"] if "membership" in o else o["changes"]
