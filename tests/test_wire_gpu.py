"""GPU parity tests of the gossip wire codec through the C ABI (rp_wire_encode_dev /
rp_wire_decode_dev and their host-buffer and first-round forms): change records as
dissemination.js:163-170 / 64-73 emit them (undefined members left out per record), wrapped as
the ping (ping-sender.js:71-76, ping.js:45-48), ping-req (ping-req-sender.js:75-81,
ping-req.js:61-65) and join response (join.js:128-133) bodies.

Oracle: tests/golden/wire_golden.json (the reference's Dissemination run in node) and
oracle/pywire.py (pinned against it in tests/test_oracle_wire.py). Bit-exact bytes.
"""
import json
import os
import random
import sys
import uuid

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import pywire  # noqa: E402
import wire_texts as wt  # noqa: E402

ST = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}
NULL = 0xFFFFFFFF
INT64_MIN = -(2 ** 63)


def golden():
    with open(os.path.join(HERE, "golden", "wire_golden.json")) as f:
        return json.load(f)["cases"]


def split(blob, off):
    return [blob[int(off[j]):int(off[j + 1])].decode() for j in range(len(off) - 1)]


def encode_cases(gpu, m, cases, form, body, app=None):
    rec_off, addr, src, st, inc, sinc, ids = [0], [], [], [], [], [], []
    cks, msrc, msinc, tgt, pst = [], [], [], [], []
    for c in cases:
        if form == "issueAs":
            rows = [(ch[0], ch[3], ch[1], ch[2], ch[4], ch[5]) for ch in c["changes"]]
        else:
            rows = [(mm[0], c["whoami"], mm[1], mm[2], None, None) for mm in c["members"]]
        for a, s_, status, i_, si, id_ in rows:
            addr.append(m.intern([a])[0])
            src.append(NULL if s_ is None else m.intern([s_])[0])  # undefined source: left out
            st.append(ST[status])
            inc.append(i_)
            sinc.append(INT64_MIN if si is None else si)
            ids.append(np.frombuffer(id_.encode(), dtype=np.uint8) if id_ else np.zeros(36, np.uint8))
        rec_off.append(len(addr))
        cks.append(c["checksum"])
        msrc.append(m.intern([c["whoami"]])[0])
        msinc.append(c["whoamiInc"])
        tgt.append(m.intern([c["target"]])[0])
        pst.append(1 if c["pingStatus"] else 0)
    idarr = np.stack(ids) if form == "issueAs" and ids else None
    blob, off = gpu.wire_encode(m, np.array(rec_off), np.array(addr), np.array(src), np.array(st), np.array(inc),
                                np.array(sinc), idarr, form=form, body=body, msg_checksum=cks, msg_source=msrc,
                                msg_source_inc=msinc, msg_target=tgt, msg_ping_status=pst, app=app)
    return split(blob, off)


def test_encode_matches_reference_golden(gpu):
    cases = golden()
    m = gpu.Membership()
    assert any(not ch[5] for c in cases for ch in c["changes"])  # id-less records
    assert any(ch[3] is None or ch[4] is None for c in cases for ch in c["changes"])  # undefined members
    assert encode_cases(gpu, m, cases, "issueAs", "array") == [c["out"]["issueAs"] for c in cases]
    assert encode_cases(gpu, m, cases, "issueAs", "ping") == [c["out"]["ping"] for c in cases]
    assert encode_cases(gpu, m, cases, "issueAs", "pingResponse") == [c["out"]["pingResponse"] for c in cases]
    assert encode_cases(gpu, m, cases, "issueAs", "pingReq") == [c["out"]["pingReq"] for c in cases]
    assert encode_cases(gpu, m, cases, "fullSync", "array") == [c["out"]["fullSync"] for c in cases]
    for c in cases:  # the app is one string per batch
        assert encode_cases(gpu, m, [c], "fullSync", "joinResponse", app=c["app"]) == [c["out"]["joinResponse"]]


def test_encode_pingreq_response_matches_reference_golden(gpu):
    """{changes: issueAsReceiver(...), pingStatus, target} (ping-req.js:61-65): the records of the
    reference's second issueAsReceiver call (piggyback counts moved on)."""
    cases = golden()
    m = gpu.Membership()
    for c in cases:
        want = c["out"]["pingReqResponse"]
        recs = json.loads(want)["changes"]
        sub = dict(c, changes=[[r["address"], r["status"], r["incarnationNumber"], r.get("source"),
                                r.get("sourceIncarnationNumber"), r.get("id")] for r in recs])
        assert encode_cases(gpu, m, [sub], "issueAs", "pingReqResponse") == [want]


def test_encode_rejects_bad_ids_and_offsets(gpu):
    """An id the name table does not hold (e.g. RP_NULL_ID from decoding an un-interned
    address) or offsets that do not start at 0 / decrease are a clean RP_EINVAL, never a device
    out-of-bounds read."""
    m = gpu.Membership()
    m.intern(["10.0.0.1:1", "10.0.0.2:2"])
    ok = dict(src=np.array([0]), status=np.array([0]), inc=np.array([5]), src_inc=np.array([1]))
    with pytest.raises(gpu.RingpopAmdError, match="address"):
        gpu.wire_encode(m, np.array([0, 1]), np.array([NULL]), **ok)
    with pytest.raises(gpu.RingpopAmdError, match="source"):
        gpu.wire_encode(m, np.array([0, 1]), np.array([1]), np.array([7]), np.array([0]), np.array([5]))
    with pytest.raises(gpu.RingpopAmdError, match="offsets"):
        gpu.wire_encode(m, np.array([1, 1]), np.array([1]), **ok)
    with pytest.raises(gpu.RingpopAmdError, match="target"):
        gpu.wire_encode(m, np.array([0, 1]), np.array([1]), body="pingReqResponse", msg_target=[NULL],
                        msg_ping_status=[1], **ok)
    blob, _ = gpu.wire_encode(m, np.array([0, 1]), np.array([1]), **ok)
    assert blob == b'[{"source":"10.0.0.1:1","sourceIncarnationNumber":1,"address":"10.0.0.2:2",' \
                   b'"status":"alive","incarnationNumber":5}]'


def test_decode_reference_golden(gpu):
    cases = golden()
    m = gpu.Membership()
    for c in cases:
        m.intern([mm[0] for mm in c["members"]])
    kinds = ["ping", "issueAs", "pingResponse", "fullSync", "pingReq", "pingReqResponse", "joinResponse"]
    K = len(kinds)
    texts = []
    for c in cases:
        texts += [c["out"][x] for x in kinds]
    d = gpu.wire_decode(m, texts)
    assert (d["err"] == 0).all()
    for j, t in enumerate(texts):
        want = pywire.decode(t)
        a, b = int(d["rec_off"][j]), int(d["rec_off"][j + 1])
        assert b - a == len(want)
        raw = t.encode()
        for k, w in zip(range(a, b), want):
            assert m.address(int(d["addr"][k])) == w["address"]
            assert (m.address(int(d["src"][k])) if int(d["src"][k]) != NULL else None) == w.get("source")
            assert int(d["status"][k]) == ST[w["status"]]
            assert int(d["inc"][k]) == w["incarnationNumber"]
            assert int(d["src_inc"][k]) == w.get("sourceIncarnationNumber", INT64_MIN)
            if "id" in w:
                o = int(d["id_off"][k]) - int(sum(len(x.encode()) for x in texts[:j]))
                assert raw[o:o + 36].decode() == w["id"]
            else:
                assert int(d["id_off"][k]) == 2 ** 64 - 1
    # body headers: ping (ping.js:27-36), ping-req request / response, join response
    for i, c in enumerate(cases):
        j = K * i
        assert int(d["checksum"][j]) == c["checksum"]
        assert m.address(int(d["source"][j])) == c["whoami"]
        assert int(d["source_inc"][j]) == c["whoamiInc"]
        assert int(d["ping_status"][j]) == 0xFF and int(d["target"][j]) == NULL
        assert m.address(int(d["target"][j + 4])) == c["target"] and int(d["source_inc"][j + 4]) == c["whoamiInc"]
        assert int(d["ping_status"][j + 5]) == (1 if c["pingStatus"] else 0)
        assert m.address(int(d["target"][j + 5])) == c["target"]
        assert m.address(int(d["source"][j + 6])) == c["whoami"]  # coordinator
        assert int(d["checksum"][j + 6]) == c["checksum"]  # membershipChecksum


def test_decode_tolerates_json_layout_and_flags_errors(gpu):
    m = gpu.Membership()
    m.intern(["10.0.0.1:1", "10.0.0.2:2"])
    texts = [
        ' { "changes" : [ {"status":"faulty", "extra":{"a":[1,{"b":"]"}]}, "incarnationNumber": 7,'
        ' "address":"10.0.0.2:2"} ] , "checksum": 5 }\n',
        '[{"address":"10.0.0.9:9","status":"alive","incarnationNumber":-3}]',  # not interned
        '[]',
        '[{"address":"10.0.0.1:1","status":"dead","incarnationNumber":1}]',  # bad status
        '[{"address":"10.0.0.1:1","status":"alive","incarnationNumber":1.5}]',  # non-integral
        '[{"address":"10.0\\u002e0.1:1","status":"alive","incarnationNumber":1}]',  # escape
        '[{"address":"10.0.0.1:1","status":"alive"}]',  # missing incarnationNumber
        '{"checksum":1}',  # no changes
        '[{"address":"10.0.0.1:1","status":"leave","incarnationNumber":2}',  # truncated
        '[{"address":"10.0.0.1:1","status":"leave","incarnationNumber":2}] x',  # trailing bytes
        '',
    ]
    d = gpu.wire_decode(m, texts)
    ok = [int(e) == 0 for e in d["err"]]
    assert ok == [True, True, True] + [False] * 8
    ro = d["rec_off"]
    assert list(np.diff(ro)) == [1, 1, 0] + [0] * 8
    assert m.address(int(d["addr"][0])) == "10.0.0.2:2" and int(d["status"][0]) == 2 and int(d["inc"][0]) == 7
    assert int(d["src"][0]) == NULL and int(d["checksum"][0]) == 5
    assert int(d["addr"][1]) == NULL and int(d["inc"][1]) == -3
    o, n = int(d["addr_off"][1]), int(d["addr_len"][1])
    base = len(texts[0].encode())
    assert (texts[0] + texts[1]).encode()[o:o + n] == b"10.0.0.9:9" and o > base


@pytest.mark.parametrize("n_msgs,max_recs", [(1, 0), (3000, 40), (20000, 90)])
def test_round_trip_large(gpu, n_msgs, max_recs):
    """encode -> decode identity at gossip scale, plus the oracle's bytes on a sample."""
    rng = np.random.default_rng(n_msgs)
    names = ["10.%d.%d.%d:%d" % (i >> 16, (i >> 8) & 255, i & 255, 3000 + i % 997) for i in range(5000)]
    m = gpu.Membership()
    m.intern(names)
    counts = rng.integers(0, max_recs + 1, n_msgs)
    rec_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    k = int(rec_off[-1])
    addr = rng.integers(0, len(names), k).astype(np.uint32)
    src = rng.integers(0, len(names), k).astype(np.uint32)
    st = rng.integers(0, 4, k).astype(np.uint8)
    inc = rng.integers(-5, 2 ** 53, k).astype(np.int64)
    sinc = rng.integers(0, 2 ** 53, k).astype(np.int64)
    pyr = random.Random(n_msgs)
    ids_s = [str(uuid.UUID(int=pyr.getrandbits(128), version=4)) for _ in range(k)]
    ids = np.frombuffer("".join(ids_s).encode(), dtype=np.uint8).reshape(k, 36) if k else None
    blob, off = gpu.wire_encode(m, rec_off, addr, src, st, inc, sinc, ids)
    texts = split(blob, off)
    for j in sorted(set(rng.integers(0, n_msgs, 50).tolist())):
        recs = [pywire.issue_as_record(ids_s[r], names[src[r]], int(sinc[r]), names[addr[r]],
                                       pywire.STATUS_NAME[st[r]], int(inc[r])) for r in range(rec_off[j], rec_off[j + 1])]
        assert texts[j] == pywire.body(recs)
    d = gpu.wire_decode(m, texts)
    assert (d["err"] == 0).all()
    assert (d["rec_off"] == rec_off).all()
    assert (d["addr"] == addr).all() and (d["src"] == src).all() and (d["status"] == st).all()
    assert (d["inc"] == inc).all() and (d["src_inc"] == sinc).all()


def test_host_buffer_forms_match_device_forms(gpu):
    """rp_wire_encode_changes / rp_wire_decode_changes (host buffers) == the _dev forms."""
    import ctypes
    cases = golden()
    m = gpu.Membership()
    c = cases[2]
    want = encode_cases(gpu, m, [c], "issueAs", "ping")[0]
    L = gpu.lib()
    ro = np.array([0, len(c["changes"])], dtype=np.uint32)
    addr = np.array(m.intern([ch[0] for ch in c["changes"]]), dtype=np.uint32)
    src = np.array(m.intern([ch[3] for ch in c["changes"]]), dtype=np.uint32)
    st = np.array([ST[ch[1]] for ch in c["changes"]], dtype=np.uint8)
    inc = np.array([ch[2] for ch in c["changes"]], dtype=np.int64)
    sinc = np.array([ch[4] for ch in c["changes"]], dtype=np.int64)
    ids = np.frombuffer("".join(ch[5] for ch in c["changes"]).encode(), dtype=np.uint8).copy()
    ck = np.array([c["checksum"]], dtype=np.uint32)
    ms = np.array(m.intern([c["whoami"]]), dtype=np.uint32)
    msi = np.array([c["whoamiInc"]], dtype=np.int64)
    off = np.zeros(2, dtype=np.uint64)
    args = [m._h, 1, ro.ctypes.data, addr.ctypes.data, src.ctypes.data, st.ctypes.data, inc.ctypes.data,
            sinc.ctypes.data, ids.ctypes.data, 0, 1, ck.ctypes.data, ms.ctypes.data, msi.ctypes.data]
    gpu.check(L.rp_wire_encode_changes(*args, None, 0, off.ctypes.data))
    out = np.zeros(int(off[1]), dtype=np.uint8)
    assert L.rp_wire_encode_changes(*args, out.ctypes.data, len(out) - 1, off.ctypes.data) != 0  # too small
    gpu.check(L.rp_wire_encode_changes(*args, out.ctypes.data, len(out), off.ctypes.data))
    assert out.tobytes().decode() == want == c["out"]["ping"]
    texts = [want.encode(), b"[", c["out"]["fullSync"].encode()]
    moff = np.concatenate([[0], np.cumsum([len(t) for t in texts])]).astype(np.uint64)
    blob = b"".join(texts)
    cap = 1000
    rro = np.zeros(4, dtype=np.uint32)
    a2, s2 = np.zeros(cap, dtype=np.uint32), np.zeros(cap, dtype=np.uint32)
    st2, i2, si2 = np.zeros(cap, dtype=np.uint8), np.zeros(cap, dtype=np.int64), np.zeros(cap, dtype=np.int64)
    err = np.zeros(3, dtype=np.uint64)
    m.intern([mm[0] for mm in c["members"]])
    gpu.check(L.rp_wire_decode_changes(m._h, blob, moff.ctypes.data, 3, rro.ctypes.data, cap, a2.ctypes.data,
                                       s2.ctypes.data, st2.ctypes.data, i2.ctypes.data, si2.ctypes.data,
                                       err.ctypes.data))
    assert err[0] == 0 and err[1] != 0 and err[2] == 0
    k = len(c["changes"])
    assert list(np.diff(rro)) == [k, 0, len(c["members"])]
    assert (a2[:k] == addr).all() and (s2[:k] == src).all() and (st2[:k] == st).all() and (i2[:k] == inc).all()
    assert (si2[:k] == sinc).all()
    fs = pywire.decode(c["out"]["fullSync"])
    assert [m.address(int(x)) for x in a2[k:k + len(fs)]] == [r["address"] for r in fs]


def test_host_buffer_full_api(gpu):
    """rp_wire_encode / rp_wire_decode (host buffers, record + header structs): a ping-req
    request round trip with an address that is not interned yet — the host decode hands back its
    bytes (addr_off / addr_len) and every header column."""
    import ctypes
    m = gpu.Membership()
    names = ["10.0.0.%d:1" % i for i in range(5)]
    ids = np.array(m.intern(names), dtype=np.uint32)
    L = gpu.lib()
    ro = np.array([0, 2], dtype=np.uint32)
    addr, src = ids[[1, 2]].copy(), np.array([ids[3], gpu.NULL_ID], dtype=np.uint32)
    st, inc = np.array([1, 3], dtype=np.uint8), np.array([7, 9], dtype=np.int64)
    sinc = np.array([11, gpu.INT64_MIN], dtype=np.int64)
    ck, ms, msi, tg = (np.array([x], dtype=dt) for x, dt in ((99, np.uint32), (ids[0], np.uint32), (5, np.int64),
                                                            (ids[4], np.uint32)))
    P = lambda a: a.ctypes.data  # noqa: E731
    recs = gpu.WireRecords(P(addr), P(src), P(st), P(inc), P(sinc), None)
    hdr = gpu.WireHeaders(P(ck), P(ms), P(msi), P(tg), None, None, 0)
    off = np.zeros(2, dtype=np.uint64)
    gpu.check(L.rp_wire_encode(m._h, 1, P(ro), ctypes.byref(recs), 0, 3, ctypes.byref(hdr), None, 0, P(off)))
    out = np.zeros(int(off[1]), dtype=np.uint8)
    gpu.check(L.rp_wire_encode(m._h, 1, P(ro), ctypes.byref(recs), 0, 3, ctypes.byref(hdr), P(out), len(out), P(off)))
    text = out.tobytes().decode()
    assert json.loads(text) == {"checksum": 99, "changes": [
        {"source": names[3], "sourceIncarnationNumber": 11, "address": names[1], "status": "suspect",
         "incarnationNumber": 7},
        {"address": names[2], "status": "leave", "incarnationNumber": 9}],
        "source": names[0], "sourceIncarnationNumber": 5, "target": names[4]}
    text2 = text.replace(names[2], "10.9.9.9:9")  # not interned
    blob = text2.encode()
    moff = np.array([0, len(blob)], dtype=np.uint64)
    cap = 8
    cols = dict(addr=np.zeros(cap, np.uint32), src=np.zeros(cap, np.uint32), status=np.zeros(cap, np.uint8),
                inc=np.zeros(cap, np.int64), src_inc=np.zeros(cap, np.int64), id_off=np.zeros(cap, np.uint64),
                addr_off=np.zeros(cap, np.uint64), addr_len=np.zeros(cap, np.uint32))
    hcols = dict(checksum=np.zeros(1, np.uint32), source=np.zeros(1, np.uint32), source_inc=np.zeros(1, np.int64),
                 target=np.zeros(1, np.uint32), ping_status=np.zeros(1, np.uint8))
    ro2, err = np.zeros(2, np.uint32), np.zeros(1, np.uint64)
    rout = gpu.WireRecordsOut(*[P(cols[k]) for k in ("addr", "src", "status", "inc", "src_inc", "id_off", "addr_off",
                                                     "addr_len")])
    hout = gpu.WireHeadersOut(*[P(hcols[k]) for k in ("checksum", "source", "source_inc", "target", "ping_status")])
    gpu.check(L.rp_wire_decode(m._h, blob, P(moff), 1, P(ro2), cap, ctypes.byref(rout), ctypes.byref(hout), P(err)))
    assert err[0] == 0 and ro2[1] == 2
    assert cols["addr"][0] == ids[1] and cols["addr"][1] == gpu.NULL_ID
    o, n = int(cols["addr_off"][1]), int(cols["addr_len"][1])
    assert blob[o:o + n] == b"10.9.9.9:9"
    assert cols["src"][1] == gpu.NULL_ID and cols["src_inc"][1] == gpu.INT64_MIN and cols["src_inc"][0] == 11
    assert (hcols["checksum"][0], hcols["source"][0], hcols["source_inc"][0], hcols["target"][0],
            hcols["ping_status"][0]) == (99, ids[0], 5, ids[4], 0xFF)
    # host decode: null buffer with bytes is an error, not a read past a 1-byte buffer
    assert L.rp_wire_decode(m._h, None, P(moff), 1, P(ro2), cap, ctypes.byref(rout), None, P(err)) != 0


@pytest.mark.parametrize("grid", [None, "3"], ids=["wave-per-message", "waves-stride-messages"])
def test_wave_decoder_equals_thread_decoder(gpu, monkeypatch, capfd, grid):
    """The wave-per-message decoder (k_decode_wave) and the thread parser (RP_WIRE_THREAD=1)
    return the contract's columns (oracle/pywire.decode_columns: errors and their offsets,
    records, headers) on the reference's bodies, re-laid-out variants with unknown members, and
    single-character mutants, and identical columns to one another; the waves take every
    well-formed message. grid "3": three workgroups, so every wave parses many messages one after
    another in the same LDS (RP_WIRE_GRID)."""
    cases = wt.golden()
    m = gpu.Membership()
    ids = wt.name_ids(m, wt.golden_names(cases))
    texts = wt.fuzz_texts(cases, 11)
    if grid:
        monkeypatch.setenv("RP_WIRE_GRID", grid)
    monkeypatch.setenv("RP_WIRE_DEBUG", "1")
    capfd.readouterr()
    dw = gpu.wire_decode(m, texts)
    err = capfd.readouterr().err
    wt.check_against_contract(dw, texts, ids, "waves")
    monkeypatch.setenv("RP_WIRE_THREAD", "1")
    dt = gpu.wire_decode(m, texts)
    wt.check_against_contract(dt, texts, ids, "thread")
    for k in dt:
        assert np.array_equal(dw[k], dt[k]), k
    n_ok = int((dt["err"] == 0).sum())
    assert n_ok > 120 and n_ok < len(texts)
    line = [x for x in err.splitlines() if "by waves" in x][-1]
    by_waves = int(line.split()[3])
    big = sum(1 for t in texts if len(t.encode()) > 8192)
    assert by_waves >= n_ok - big, line


@pytest.mark.parametrize("thread", [False, True], ids=["waves", "thread-parser"])
def test_decode_name_lengths_around_the_inline_prefix(gpu, monkeypatch, thread):
    """The decoder's name index keeps a name's first 20 bytes in its hash slot and reads only
    the rest from the name bytes: interned names of 0..70 bytes, names sharing their first 20
    bytes (and more) with one another, and strings that are a prefix or an extension of an
    interned name by one byte (not interned: NULL id). Records' address / source and the body's
    source and target go through the same lookup."""
    rng = random.Random(3)
    base = "".join(rng.choice("0123456789abcdef.:") for _ in range(70))
    names = sorted({base[:n] for n in range(1, 71)} | {base[:20] + "x" + base[21:n] for n in range(21, 40)} |
                   {"10.0.%d.%d:%d" % (i, i * 7 % 256, 3000 + i) for i in range(40)} |
                   {"".join(rng.choice("abc") for _ in range(rng.randrange(1, 64))) for _ in range(200)})
    m = gpu.Membership()
    ids = dict(zip(names, m.intern(names)))
    probes = names + [n + "q" for n in names[:60]] + [n[:-1] for n in names[:60] if len(n) > 1]
    rng.shuffle(probes)
    texts = []
    want_addr, want_src, want_hsrc, want_tgt = [], [], [], []
    for i in range(0, len(probes), 5):
        chunk = probes[i:i + 5]
        recs = []
        for j, a in enumerate(chunk):
            s = chunk[(j + 1) % len(chunk)]
            recs.append({"address": a, "status": "alive", "incarnationNumber": 7, "source": s})
            want_addr.append(ids.get(a, NULL))
            want_src.append(ids.get(s, NULL))
        hs, tg = chunk[0], chunk[-1]
        want_hsrc.append(ids.get(hs, NULL))
        want_tgt.append(ids.get(tg, NULL))
        texts.append(json.dumps({"checksum": 1, "changes": recs, "source": hs, "sourceIncarnationNumber": 2,
                                 "target": tg}, separators=(",", ":")))
    if thread:
        monkeypatch.setenv("RP_WIRE_THREAD", "1")
    d = gpu.wire_decode(m, texts)
    assert (d["err"] == 0).all()
    assert d["addr"].tolist() == want_addr
    assert d["src"].tolist() == want_src
    assert d["source"].tolist() == want_hsrc
    assert d["target"].tolist() == want_tgt
    wt.check_against_contract(d, texts, {n.encode(): int(i) for n, i in ids.items()}, "names")
    m.close()


def test_two_pass_layouts_match_thread_parser(gpu, monkeypatch, capfd):
    """The wave decoder's first pass holds 1,280 tokens a message; longer token lists are left to
    the second pass (2,048 tokens), past that to the thread parser. Changes arrays of 40..120 short
    records (about 740 to 2,180 tokens in under 8 KB) decode to the contract's columns through both
    passes, the full layout alone (RP_WIRE_ONEPASS=1) and the thread parser, and the waves take
    every message of at most 2,048 tokens."""
    names, texts = wt.long_array_texts()
    m = gpu.Membership()
    ids = wt.name_ids(m, names)
    toks = [wt.count_tokens(t) for t in texts]
    assert min(toks) < 1280 < max(toks) and max(toks) > 2048 and any(1280 < x <= 2048 for x in toks)
    assert all(len(t) <= 8192 for t in texts)
    monkeypatch.setenv("RP_WIRE_DEBUG", "1")
    capfd.readouterr()
    d2 = gpu.wire_decode(m, texts)
    line = [x for x in capfd.readouterr().err.splitlines() if "by waves" in x][-1]
    assert int(line.split()[3]) == sum(1 for x in toks if x <= 2048), line
    monkeypatch.setenv("RP_WIRE_ONEPASS", "1")
    d1 = gpu.wire_decode(m, texts)
    monkeypatch.delenv("RP_WIRE_ONEPASS")
    monkeypatch.setenv("RP_WIRE_THREAD", "1")
    dt = gpu.wire_decode(m, texts)
    for what, d in (("two-pass", d2), ("one-pass", d1), ("thread", dt)):
        wt.check_against_contract(d, texts, ids, what)
    for k in dt:
        assert np.array_equal(d2[k], dt[k]), k
        assert np.array_equal(d1[k], dt[k]), k
    assert (dt["err"] == 0).all()
    m.close()


def test_messages_past_the_first_pass_bytes(gpu, monkeypatch, capfd):
    """Messages of 7.2-8 KB with fewer than 1,280 tokens (long addresses, sources, ids and an
    unknown padding string; some addresses not interned) leave the first pass for its 7 KB byte
    buffer, not its token count: the default two-pass layout, the full layout alone
    (RP_WIRE_ONEPASS=1) and the thread parser all give the contract's columns, and the waves take
    every message."""
    names, texts = wt.big_byte_texts()
    m = gpu.Membership()
    ids = wt.name_ids(m, names)
    assert all(7168 < len(t) <= 8192 for t in texts) and all(wt.count_tokens(t) < 1280 for t in texts)
    monkeypatch.setenv("RP_WIRE_DEBUG", "1")
    capfd.readouterr()
    d2 = gpu.wire_decode(m, texts)
    line = [x for x in capfd.readouterr().err.splitlines() if "by waves" in x][-1]
    assert int(line.split()[3]) == len(texts), line
    monkeypatch.setenv("RP_WIRE_ONEPASS", "1")
    d1 = gpu.wire_decode(m, texts)
    monkeypatch.delenv("RP_WIRE_ONEPASS")
    monkeypatch.setenv("RP_WIRE_THREAD", "1")
    dt = gpu.wire_decode(m, texts)
    for what, d in (("two-pass", d2), ("one-pass", d1), ("thread", dt)):
        wt.check_against_contract(d, texts, ids, what)
    assert (dt["err"] == 0).all() and int(dt["rec_off"][-1]) > 10 * len(texts)
    m.close()


def test_bodies_past_64_members_take_the_serial_walk(gpu, monkeypatch, capfd):
    """The body's members are parsed a lane each up to 64 members; a body with more (unknown
    members around the known ones, a repeated source) takes the wave-uniform serial walk. Both
    give the contract's columns and headers (and the thread parser's), and the waves take every
    such message."""
    names, texts = wt.many_member_texts()
    m = gpu.Membership()
    ids = wt.name_ids(m, names)
    monkeypatch.setenv("RP_WIRE_DEBUG", "1")
    capfd.readouterr()
    dw = gpu.wire_decode(m, texts)
    line = [x for x in capfd.readouterr().err.splitlines() if "by waves" in x][-1]
    assert int(line.split()[3]) == len(texts), line
    wt.check_against_contract(dw, texts, ids, "waves")
    monkeypatch.setenv("RP_WIRE_THREAD", "1")
    dt = gpu.wire_decode(m, texts)
    wt.check_against_contract(dt, texts, ids, "thread")
    for k in dt:
        assert np.array_equal(dw[k], dt[k]), k
    assert (dt["err"] == 0).all() and (dt["source"] == m.intern([names[2]])[0]).all()
    m.close()
