"""Wire-decoder test inputs and the contract check shared by the CPU oracle tests
(test_oracle_wire.py) and the GPU parity tests (test_wire_gpu.py).

The texts: the reference's bodies (tests/golden/wire_golden.json) re-laid-out with unknown
members and single-character mutants; long changes arrays around the decoder's token limits;
bodies with many members; messages of 7.2-8 KB with few tokens. The check compares decoded
columns with oracle/pywire.decode_columns (the decoder's contract restated on the CPU)."""
import json
import os
import random

import numpy as np

import pywire

HERE = os.path.dirname(os.path.abspath(__file__))
ST = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}
KINDS = ["ping", "issueAs", "pingResponse", "fullSync", "pingReq", "pingReqResponse", "joinResponse"]


def golden():
    with open(os.path.join(HERE, "golden", "wire_golden.json")) as f:
        return json.load(f)["cases"]


def golden_names(cases):
    return sorted({mm[0] for c in cases for mm in c["members"]} | {c["target"] for c in cases})


def fuzz_texts(cases, seed):
    """The reference's bodies re-serialised with random layouts and unknown members, then a set of
    single-character mutations (most of them invalid JSON)."""
    rng = random.Random(seed)
    base = [c["out"][k] for c in cases for k in KINDS]
    ws = [" ", "\n", "\t", "\r\n ", ""]

    def shuffle(o):
        if isinstance(o, dict):
            items = [(k, shuffle(v)) for k, v in o.items()]
            rng.shuffle(items)
            if rng.random() < 0.3:
                items.insert(rng.randrange(len(items) + 1), ("x%d" % rng.randrange(9), rng.choice(
                    [None, True, False, -12, "s:t[r]{,}", [1, {"b": "]"}, []], {"a": {"c": [None]}}, 3.5e2])))
            return dict(items)
        if isinstance(o, list):
            return [shuffle(v) for v in o]
        return o

    out = []
    for t in base:
        out.append(t)
        o = json.loads(t)
        for _ in range(2):
            sep = (rng.choice(ws) + "," + rng.choice(ws), rng.choice(ws) + ":" + rng.choice(ws))
            out.append(rng.choice(ws) + json.dumps(shuffle(o), separators=sep) + rng.choice(ws))
    mutants = []
    for t in rng.sample(out, min(len(out), 400)):
        if not t:
            continue
        i = rng.randrange(len(t))
        kind = rng.randrange(9)
        if kind == 0:
            mutants.append(t[:i] + t[i + 1:])  # delete
        elif kind == 1:
            mutants.append(t[:i] + rng.choice('{}[]:,"\\ \t0a-.e\x01') + t[i:])  # insert
        elif kind == 2:
            mutants.append(t[:i])  # truncate
        elif kind == 3:
            mutants.append(t.replace("}", ",}", 1))  # trailing comma
        elif kind == 4:
            mutants.append(t.replace('"status"', '"status":"alive","status"', 1))  # duplicate key
        elif kind == 5:
            mutants.append(t + rng.choice([" ", "x", "]", ",", "{}"]))  # trailing bytes
        elif kind == 6:  # a repeated body key: the last one wins
            mutants.append(t.replace('"source"', '"source":"%s","source"' % rng.choice(["x", "127.0.0.1:3001"]), 1))
        elif kind == 7:
            mutants.append(t.replace('"checksum"', '"checksum":5,"checksum"', 1))
        else:  # a repeated changes array
            mutants.append(t.replace('"changes"', '"changes":[],"changes"', 1))
    return out + mutants


def count_tokens(t):
    """Quotes and the structural characters outside strings (the wave decoder's tokens)."""
    n, ins, esc = 0, False, False
    for ch in t:
        if ins:
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                ins = False
                n += 1
        elif ch == '"':
            ins = True
            n += 1
        elif ch in "{}[]:,":
            n += 1
    return n


def long_array_texts():
    """Changes arrays of 40..120 short records (about 740 to 2,180 tokens in under 8 KB)."""
    rng = random.Random(9)
    names = ["n%d" % i for i in range(200)]
    texts = []
    for k in range(40, 124, 4):
        recs = [{"address": rng.choice(names + ["zz%d" % k]), "status": rng.choice(list(ST)),
                 "incarnationNumber": rng.randrange(10 ** 6)} for _ in range(k)]
        texts.append(json.dumps({"checksum": k, "changes": recs, "source": names[k], "sourceIncarnationNumber": 1},
                                separators=(",", ":")))
    return names, texts


def many_member_texts():
    """Bodies with 0..90 unknown members around the known ones and a repeated source."""
    rng = random.Random(5)
    names = ["10.0.0.%d:3000" % i for i in range(40)]
    texts = []
    for nextra in (0, 30, 62, 63, 64, 65, 90):
        body = [("checksum", 7), ("source", names[1]), ("sourceIncarnationNumber", 3)]
        body += [("x%d" % j, [1, {"a": 1}] if j % 9 == 4 else rng.choice([1, "s", None, True])) for j in range(nextra)]
        body.insert(rng.randrange(len(body) + 1), ("changes", [{"address": rng.choice(names), "status": "alive",
                                                                 "incarnationNumber": j} for j in range(5)]))
        body.append(("source", names[2]))  # the last repeated key wins
        texts.append("{" + ",".join(json.dumps(k) + ":" + json.dumps(v) for k, v in body) + "}")
    return names, texts


def big_byte_texts():
    """Messages of 7.2-8 KB with fewer than 1,280 tokens (long address / source / id strings and
    long unknown strings): past the first pass's 7 KB byte buffer, within the second pass's
    (the byte-length handoff had no test of its own)."""
    rng = random.Random(21)
    names = ["host-%s.example.internal:%d" % ("".join(rng.choice("abcdefgh") for _ in range(rng.randrange(60, 200))),
                                               3000 + i) for i in range(40)]
    texts = []
    for target in range(7200, 8192, 90):
        recs = []
        body = {"checksum": target, "changes": recs, "source": names[0], "sourceIncarnationNumber": 9}
        while True:
            r = {"id": "%08x-0000-4000-8000-%012x" % (rng.getrandbits(32), rng.getrandbits(48)),
                 "source": rng.choice(names), "sourceIncarnationNumber": rng.randrange(10 ** 12),
                 "address": rng.choice(names + ["not-interned-%d.example:1" % len(recs)]),
                 "status": rng.choice(list(ST)), "incarnationNumber": rng.randrange(10 ** 12)}
            recs.append(r)
            if len(json.dumps(body, separators=(",", ":"))) > target - 600:
                break
        t = json.dumps(body, separators=(",", ":"))
        pad = target - len(t) - len(',"pad":""')
        if pad > 0:
            t = t[:-1] + ',"pad":"' + "p" * pad + '"}'
        texts.append(t)
    return names, texts


def check_against_contract(d, texts, ids, what=""):
    """Every column of a decode (gpu.wire_decode's dict) equals the contract's
    (pywire.decode_columns): errors and their offsets, record counts, addresses, sources,
    statuses, incarnation numbers, id / address byte offsets, and, for messages without an error,
    the header columns."""
    base = 0
    ro = d["rec_off"]
    for j, t in enumerate(texts):
        b = t.encode() if isinstance(t, str) else bytes(t)
        w = pywire.decode_columns(b, ids)
        assert int(d["err"][j]) == w["err"], (what, j, int(d["err"][j]), w["err"], t[:200])
        a, e = int(ro[j]), int(ro[j + 1])
        assert e - a == len(w["records"]), (what, j)
        for k, r in zip(range(a, e), w["records"]):
            assert int(d["addr"][k]) == r["addr"], (what, j, k)
            assert int(d["src"][k]) == r["src"], (what, j, k)
            assert int(d["status"][k]) == r["status"], (what, j, k)
            assert int(d["inc"][k]) == r["inc"], (what, j, k)
            assert int(d["src_inc"][k]) == r["src_inc"], (what, j, k)
            assert int(d["id_off"][k]) == (2 ** 64 - 1 if r["id_off"] is None else base + r["id_off"]), (what, j, k)
            assert int(d["addr_off"][k]) == base + r["addr_off"], (what, j, k)
            assert int(d["addr_len"][k]) == r["addr_len"], (what, j, k)
        if w["err"] == 0:
            for col in ("checksum", "source", "source_inc", "target", "ping_status"):
                assert int(d[col][j]) == w[col], (what, j, col)
        base += len(b)


def name_ids(m, names):
    """The id map of interned names (intern is idempotent: it returns the existing ids)."""
    names = list(names)
    return {n.encode(): int(i) for n, i in zip(names, m.intern(names))}


class _Int(int):
    digits = 0


class _Float(float):
    pass


class _Pairs(list):
    pass


def _int_tok(s):
    v = _Int(int(s))
    v.digits = len(s.lstrip("-"))
    return v


def json_contract(text, ids):
    """What json.loads makes of a message under the decoder's contract: None when json.loads
    rejects it; otherwise {ok, records, headers} where ok says whether the contract accepts it
    (strings without escapes; known numbers integral with at most 18 digits; known members of the
    right JSON type; address, status and incarnationNumber in every record; a changes array
    present) and the columns are read from the parsed pairs in order (a repeated member: the last
    one wins; `membership` / `membershipChecksum` / `coordinator` alias their ping names)."""
    try:
        o = json.loads(text, object_pairs_hook=_Pairs, parse_int=_int_tok, parse_float=_Float)
    except ValueError:
        return None
    nid = lambda s: ids.get(s.encode(), pywire.NULL_ID)  # noqa: E731
    is_int = lambda v: isinstance(v, _Int) and v.digits <= 18  # noqa: E731
    res = dict(ok=True, records=[], checksum=0, source=pywire.NULL_ID, source_inc=pywire.INT64_MIN,
               target=pywire.NULL_ID, ping_status=0xFF)

    def bad():
        res["ok"] = False

    def record(r):
        if not isinstance(r, _Pairs):
            return bad()
        c = dict(addr=None, src=pywire.NULL_ID, status=None, inc=None, src_inc=pywire.INT64_MIN, id=None)
        for k, v in r:
            if k == "address":
                if not isinstance(v, str):
                    return bad()
                c["addr"] = v
            elif k == "source":
                if not isinstance(v, str):
                    return bad()
                c["src"] = nid(v)
            elif k == "status":
                if v not in ST:
                    return bad()
                c["status"] = ST[v]
            elif k in ("incarnationNumber", "sourceIncarnationNumber"):
                if not is_int(v):
                    return bad()
                c["inc" if k == "incarnationNumber" else "src_inc"] = int(v)
            elif k == "id":
                if not isinstance(v, str):
                    return bad()
                c["id"] = v
        if not c["addr"] or c["status"] is None or c["inc"] is None:
            return bad()
        c["addr_name"], c["addr"] = c["addr"], nid(c["addr"])
        res["records"].append(c)

    def changes(v):
        if not isinstance(v, list) or isinstance(v, _Pairs):
            return bad()
        res["records"] = []
        for r in v:
            record(r)

    if "\\" in text:
        bad()
    if isinstance(o, list) and not isinstance(o, _Pairs):
        changes(o)
    elif isinstance(o, _Pairs):
        seen = False
        for k, v in o:
            if k in ("changes", "membership"):
                changes(v)
                seen = True
            elif k in ("checksum", "membershipChecksum", "sourceIncarnationNumber"):
                if not is_int(v):
                    bad()
                elif k == "sourceIncarnationNumber":
                    res["source_inc"] = int(v)
                else:
                    res["checksum"] = int(v) & 0xFFFFFFFF
            elif k in ("source", "coordinator", "target"):
                if not isinstance(v, str):
                    bad()
                else:
                    res["target" if k == "target" else "source"] = nid(v)
            elif k == "pingStatus":
                if not isinstance(v, bool):
                    bad()
                else:
                    res["ping_status"] = int(v)
        if not seen:
            bad()
    else:
        bad()
    return res


def np_u32(x):
    return np.asarray(x, dtype=np.uint32)
