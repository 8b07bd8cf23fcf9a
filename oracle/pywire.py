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


# ---------------------------------------------------------------- the decoder's contract
# rp_wire_decode* (include/ringpop_amd.h, "Decode n_msgs JSON texts"): the columns the device
# decoder must return for one message, restated as a recursive descent over the bytes. The
# members read are those of server/protocol/ping.js:27-36 (`changes`, `checksum`, `source`,
# `sourceIncarnationNumber`), ping-req.js:61-65 (`target`, `pingStatus`), join.js:128-133
# (`membership`, `membershipChecksum`, `coordinator`) and, per record, dissemination.js:163-170 /
# 64-73. Where the reference's JSON.parse accepts more than the contract (escapes, fractions), the
# contract rejects; unknown members are skipped by bracket depth without validating them. A
# repeated member: the last one wins (as JSON.parse). err = 0, or 1 + the byte offset at which
# the grammar first fails (the message's records are then dropped; its header columns keep the
# values read before the failure). tests/test_oracle_wire.py pins this against json.loads.

WS = b" \t\n\r"
STATUS_CODE = {b"alive": 0, b"suspect": 1, b"faulty": 2, b"leave": 3}
NULL_ID = 0xFFFFFFFF
INT64_MIN = -(2 ** 63)


class _Fail(Exception):
    pass


class _P:
    def __init__(self, b):
        self.b, self.i, self.n, self.bad_at = b, 0, len(b), None

    def fail(self):
        if self.bad_at is None:
            self.bad_at = self.i
        self.i = self.n
        raise _Fail()

    def ws(self):
        while self.i < self.n and self.b[self.i] in WS:
            self.i += 1

    def peek(self, c):
        self.ws()
        return self.i < self.n and self.b[self.i] == c

    def expect(self, c):
        if self.peek(c):
            self.i += 1
        else:
            self.fail()

    def string(self):
        """(start, length) of a string without escapes or control bytes."""
        self.ws()
        if self.i >= self.n or self.b[self.i] != 0x22:
            self.fail()
        self.i += 1
        s0 = self.i
        while self.i < self.n and self.b[self.i] != 0x22:
            if self.b[self.i] == 0x5C or self.b[self.i] < 0x20:
                self.fail()
            self.i += 1
        if self.i >= self.n:
            self.fail()
        self.i += 1
        return s0, self.i - 1 - s0

    def boolean(self):
        self.ws()
        for word, v in ((b"true", 1), (b"false", 0)):
            if self.b[self.i:self.i + len(word)] == word:
                self.i += len(word)
                return v
        self.fail()

    def integer(self):
        """An integral number of at most 18 digits (no fraction, no exponent)."""
        self.ws()
        neg = self.i < self.n and self.b[self.i] == 0x2D
        self.i += neg
        v = nd = 0
        while self.i < self.n and 0x30 <= self.b[self.i] <= 0x39:
            v = v * 10 + self.b[self.i] - 0x30
            self.i += 1
            nd += 1
            if nd > 18:
                self.fail()
        if nd == 0 or (self.i < self.n and self.b[self.i] in b".eE"):
            self.fail()
        return -v if neg else v

    def skip(self):
        """An unknown member's value: a string, a bracketed value matched by depth (strings inside
        it still without escapes), or a scalar running to the next delimiter or whitespace."""
        self.ws()
        if self.i >= self.n:
            self.fail()
        c = self.b[self.i]
        if c == 0x22:
            self.string()
        elif c in b"{[":
            depth = 0
            while self.i < self.n:
                d = self.b[self.i]
                if d == 0x22:
                    self.string()
                    continue
                if d in b"{[":
                    depth += 1
                elif d in b"}]":
                    depth -= 1
                    if depth == 0:
                        self.i += 1
                        return
                self.i += 1
            self.fail()
        else:
            while self.i < self.n and self.b[self.i] not in b",}] \n\r\t":
                self.i += 1


def _record(p, ids):
    p.expect(0x7B)
    r = dict(addr=NULL_ID, src=NULL_ID, status=None, inc=None, src_inc=INT64_MIN, id_off=None, addr_off=0, addr_len=0)
    if p.peek(0x7D):
        p.i += 1
    else:
        while True:
            ks, kl = p.string()
            p.expect(0x3A)
            key = p.b[ks:ks + kl]
            if key == b"address":
                r["addr_off"], r["addr_len"] = p.string()
                r["addr"] = ids.get(p.b[r["addr_off"]:r["addr_off"] + r["addr_len"]], NULL_ID)
            elif key == b"source":
                s, n = p.string()
                r["src"] = ids.get(p.b[s:s + n], NULL_ID)
            elif key == b"status":
                s, n = p.string()
                r["status"] = STATUS_CODE.get(p.b[s:s + n])
                if r["status"] is None:
                    p.fail()
            elif key == b"incarnationNumber":
                r["inc"] = p.integer()
            elif key == b"sourceIncarnationNumber":
                r["src_inc"] = p.integer()
            elif key == b"id":
                r["id_off"] = p.string()[0]
            else:
                p.skip()
            if p.peek(0x2C):
                p.i += 1
                continue
            p.expect(0x7D)
            break
    if r["addr_len"] == 0 or r["status"] is None or r["inc"] is None:
        p.fail()
    return r


def _changes(p, ids):
    p.expect(0x5B)
    out = []
    if p.peek(0x5D):
        p.i += 1
        return out
    while True:
        out.append(_record(p, ids))
        if p.peek(0x2C):
            p.i += 1
            continue
        p.expect(0x5D)
        return out


def decode_columns(text, ids):
    """One message's decoder columns: ids maps interned address bytes -> member id. Returns
    {err, records: [dict(addr, src, status, inc, src_inc, id_off, addr_off, addr_len)], checksum,
    source, source_inc, target, ping_status}; offsets are relative to the message."""
    b = text.encode() if isinstance(text, str) else bytes(text)
    p = _P(b)
    h = dict(checksum=0, source=NULL_ID, source_inc=INT64_MIN, target=NULL_ID, ping_status=0xFF)
    recs, seen = [], False
    try:
        if p.peek(0x5B):
            recs, seen = _changes(p, ids), True
        else:
            p.expect(0x7B)
            if p.peek(0x7D):
                p.i += 1
            else:
                while True:
                    ks, kl = p.string()
                    p.expect(0x3A)
                    key = p.b[ks:ks + kl]
                    if key in (b"changes", b"membership"):
                        recs, seen = _changes(p, ids), True
                    elif key in (b"checksum", b"membershipChecksum"):
                        h["checksum"] = p.integer() & 0xFFFFFFFF
                    elif key in (b"source", b"coordinator"):
                        s, n = p.string()
                        h["source"] = ids.get(p.b[s:s + n], NULL_ID)
                    elif key == b"sourceIncarnationNumber":
                        h["source_inc"] = p.integer()
                    elif key == b"target":
                        s, n = p.string()
                        h["target"] = ids.get(p.b[s:s + n], NULL_ID)
                    elif key == b"pingStatus":
                        h["ping_status"] = p.boolean()
                    else:
                        p.skip()
                    if p.peek(0x2C):
                        p.i += 1
                        continue
                    p.expect(0x7D)
                    break
        p.ws()
        if p.i != p.n or not seen:
            p.fail()
    except _Fail:
        recs = []
    h["err"] = 0 if p.bad_at is None else p.bad_at + 1
    h["records"] = recs
    return h
