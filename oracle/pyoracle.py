"""ctypes view of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline. The product package
(ringpop-node_amd/) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

NIL = 0xFFFFFFFF


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE, "all"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.orc_hash32.restype = ctypes.c_uint32
        L.orc_hash32.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_philox4x32_10.argtypes = [u32p, u32p, u32p]
        L.orc_uuid_key.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p]
        L.orc_gen_uuid_keys.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_c2_addr.restype = ctypes.c_int
        L.orc_c2_addr.argtypes = [ctypes.c_uint32, ctypes.c_char_p]
        L.orc_ring_new.restype = ctypes.c_void_p
        L.orc_ring_new.argtypes = [ctypes.c_uint32]
        L.orc_ring_free.argtypes = [ctypes.c_void_p]
        L.orc_ring_add_remove.restype = ctypes.c_int
        L.orc_ring_add_remove.argtypes = [ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_ring_checksum.restype = ctypes.c_int
        L.orc_ring_checksum.argtypes = [ctypes.c_void_p, u32p]
        L.orc_ring_server_count.restype = ctypes.c_uint32
        L.orc_ring_server_count.argtypes = [ctypes.c_void_p]
        L.orc_ring_token_count.restype = ctypes.c_uint32
        L.orc_ring_token_count.argtypes = [ctypes.c_void_p]
        L.orc_ring_name.restype = ctypes.c_void_p
        L.orc_ring_name.argtypes = [ctypes.c_void_p, ctypes.c_uint32, u32p]
        L.orc_ring_dump.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_ring_lookup_hash.restype = ctypes.c_uint32
        L.orc_ring_lookup_hash.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.orc_ring_lookupn_hash.restype = ctypes.c_uint32
        L.orc_ring_lookupn_hash.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p,
                                            ctypes.c_uint32]
        L.orc_ring_lookup_keys.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p]
        L.orc_ring_lookupn_keys.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_ring_lookupn_keys_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.orc_members_new.restype = ctypes.c_void_p
        L.orc_members_new.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32]
        L.orc_members_free.argtypes = [ctypes.c_void_p]
        L.orc_members_set_ready.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_members_update.restype = ctypes.c_uint32
        L.orc_members_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]
        L.orc_members_set.restype = ctypes.c_uint32
        L.orc_members_set.argtypes = [ctypes.c_void_p]
        L.orc_members_checksum.restype = ctypes.c_int
        L.orc_members_checksum.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_members_count.restype = ctypes.c_uint32
        L.orc_members_count.argtypes = [ctypes.c_void_p]
        L.orc_members_order.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_members_get.restype = ctypes.c_int
        L.orc_members_get.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_members_checksum_string.restype = ctypes.c_uint64
        L.orc_members_checksum_string.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_sim_new.restype = ctypes.c_void_p
        L.orc_sim_new.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_sim_free.argtypes = [ctypes.c_void_p]
        L.orc_sim_step.argtypes = [ctypes.c_void_p]
        L.orc_sim_round.restype = ctypes.c_int64
        L.orc_sim_round.argtypes = [ctypes.c_void_p]
        L.orc_sim_checksums.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_sim_view.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_sim_converged.restype = ctypes.c_int
        L.orc_sim_converged.argtypes = [ctypes.c_void_p]
        L.orc_sim_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_sim_event.restype = ctypes.c_int
        L.orc_sim_event.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32]
        L.orc_sim_set_threads.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_sim_piggyback.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_js_pow.restype = ctypes.c_double
        L.orc_js_pow.argtypes = [ctypes.c_double, ctypes.c_double]
        L.orc_js_round.restype = ctypes.c_double
        L.orc_js_round.argtypes = [ctypes.c_double]
        L.orc_damp_decayed.restype = ctypes.c_double
        L.orc_damp_decayed.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_int64, ctypes.c_int64]
        L.orc_damp_penalized.restype = ctypes.c_double
        L.orc_damp_penalized.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int)]
        L.orc_damp_decay_all.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p]
        _lib = L
    return _lib


def hash32(s):
    b = s.encode() if isinstance(s, str) else bytes(s)
    return lib().orc_hash32(b, len(b))


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def uuid_keys(seed, k0, n):
    """n UUID-v4-format keys as a (n, 36) uint8 array (SURVEY §8d C1/C2 key stream)."""
    buf = np.empty((n, 36), dtype=np.uint8)
    lib().orc_gen_uuid_keys(seed, k0, n, buf.ctypes.data)
    return buf


def c2_addr(i):
    b = ctypes.create_string_buffer(32)
    n = lib().orc_c2_addr(i, b)
    return b.raw[:n].decode()


def pack_strings(strs):
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strs]
    off = np.zeros(len(bs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(b) for b in bs]) if bs else []
    return b"".join(bs), off


class Ring:
    """Oracle HashRing (restates lib/ring/index.js)."""

    def __init__(self, replica_points=100):
        self.h = lib().orc_ring_new(replica_points)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_ring_free(self.h)
            self.h = None

    def add_remove(self, add=None, remove=None, add_tokens=None, rem_tokens=None):
        add = add or []
        remove = remove or []
        ab, ao = pack_strings(add)
        rb, ro = pack_strings(remove)
        at = None if add_tokens is None else np.ascontiguousarray(add_tokens, dtype=np.uint32)
        rt = None if rem_tokens is None else np.ascontiguousarray(rem_tokens, dtype=np.uint32)
        abuf = ctypes.create_string_buffer(ab, len(ab) + 1)
        rbuf = ctypes.create_string_buffer(rb, len(rb) + 1)
        return bool(lib().orc_ring_add_remove(
            self.h, abuf, ao.ctypes.data, len(add), None if at is None else at.ctypes.data,
            rbuf, ro.ctypes.data, len(remove), None if rt is None else rt.ctypes.data))

    @property
    def checksum(self):
        v = ctypes.c_uint32()
        return v.value if lib().orc_ring_checksum(self.h, ctypes.byref(v)) else None

    def server_count(self):
        return lib().orc_ring_server_count(self.h)

    def token_count(self):
        return lib().orc_ring_token_count(self.h)

    def name(self, i):
        if i == NIL:
            return None
        n = ctypes.c_uint32()
        p = lib().orc_ring_name(self.h, i, ctypes.byref(n))
        return ctypes.string_at(p, n.value).decode()

    def dump(self):
        m = self.token_count()
        t = np.empty(m, dtype=np.uint32)
        o = np.empty(m, dtype=np.uint32)
        lib().orc_ring_dump(self.h, t.ctypes.data, o.ctypes.data)
        return t, o

    def lookup_hash(self, h):
        return lib().orc_ring_lookup_hash(self.h, h)

    def lookupn_hash(self, h, n):
        cap = self.server_count() + 2
        buf = np.empty(cap, dtype=np.uint32)
        c = lib().orc_ring_lookupn_hash(self.h, h, n, buf.ctypes.data, cap)
        return [int(x) for x in buf[:c]]

    def lookup_keys(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        n, stride = keys.shape
        out = np.empty(n, dtype=np.uint32)
        lib().orc_ring_lookup_keys(self.h, keys.ctypes.data, stride, None, n, out.ctypes.data)
        return out

    def lookupn_keys(self, keys, nrep, threads=1):
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        n, stride = keys.shape
        w = max(nrep, 1)
        out = np.empty((n, w), dtype=np.uint32)
        cnt = np.empty(n, dtype=np.uint8)
        if threads > 1:
            lib().orc_ring_lookupn_keys_mt(self.h, keys.ctypes.data, stride, n, nrep, out.ctypes.data,
                                           cnt.ctypes.data, threads)
        else:
            lib().orc_ring_lookupn_keys(self.h, keys.ctypes.data, stride, None, n, nrep, out.ctypes.data,
                                        cnt.ctypes.data)
        return out, cnt


STATUS = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}
STATUS_NAME = {v: k for k, v in STATUS.items()}


class Members:
    """Oracle membership view (restates lib/membership/index.js update/set/checksum)."""

    def __init__(self, names, local=None, join_seed=0):
        self.names = list(names)
        self.index = {a: i for i, a in enumerate(self.names)}
        blob, off = pack_strings(self.names)
        self._blob = ctypes.create_string_buffer(blob, len(blob) + 1)
        lid = self.index[local] if local is not None else 0xFFFFFFFF
        self.h = lib().orc_members_new(self._blob, off.ctypes.data, len(self.names), lid, join_seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_members_free(self.h)
            self.h = None

    def set_ready(self, ready):
        lib().orc_members_set_ready(self.h, 1 if ready else 0)

    def update_ids(self, ids, status, inc, is_local=False, now_ms=0):
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        st = np.ascontiguousarray(status, dtype=np.uint8)
        inc = np.ascontiguousarray(inc, dtype=np.int64)
        k = len(ids)
        app = np.zeros(max(k, 1), dtype=np.uint8)
        nst = np.zeros(max(k, 1), dtype=np.uint8)
        ninc = np.zeros(max(k, 1), dtype=np.int64)
        n = lib().orc_members_update(self.h, ids.ctypes.data, st.ctypes.data, inc.ctypes.data, k,
                                     1 if is_local else 0, now_ms, app.ctypes.data, nst.ctypes.data,
                                     ninc.ctypes.data)
        return app[:k], nst[:k], ninc[:k], n

    def update(self, changes, is_local=False, now_ms=0):
        changes = changes if isinstance(changes, list) else [changes]
        app, nst, ninc, _ = self.update_ids([self.index[c["address"]] for c in changes],
                                            [STATUS[c["status"]] for c in changes],
                                            [c["incarnationNumber"] for c in changes], is_local, now_ms)
        out = []
        for c, a, s_, i_ in zip(changes, app, nst, ninc):
            if a:
                u = dict(c)
                u["status"] = STATUS_NAME[int(s_)]
                u["incarnationNumber"] = int(i_)
                out.append(u)
        return out

    def set(self):
        return lib().orc_members_set(self.h)

    @property
    def checksum(self):
        v = ctypes.c_uint32()
        return v.value if lib().orc_members_checksum(self.h, ctypes.byref(v)) else None

    def count(self):
        return lib().orc_members_count(self.h)

    def order(self):
        n = self.count()
        out = np.empty(max(n, 1), dtype=np.uint32)
        lib().orc_members_order(self.h, out.ctypes.data)
        return [self.names[i] for i in out[:n]]

    def member(self, address):
        st, inc = ctypes.c_uint8(), ctypes.c_int64()
        if not lib().orc_members_get(self.h, self.index[address], ctypes.byref(st), ctypes.byref(inc)):
            return None
        return {"address": address, "status": STATUS_NAME[st.value], "incarnationNumber": inc.value}

    def checksum_string(self):
        n = lib().orc_members_checksum_string(self.h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        lib().orc_members_checksum_string(self.h, buf, n)
        return buf.raw[:n].decode()


SIM_EVENT = {"kill": 0, "revive": 1, "leave": 2, "join": 3}


class Sim:
    """Oracle gossip round model (orc_sim.c). events: (round, kind, node) with kind in
    SIM_EVENT, applied before that round (a node down from round r on, back up, or leaving)."""

    def __init__(self, names, inc0, dead, seed=11, susp_rounds=25, now0=1434500000000, events=(), threads=None):
        self.N = len(names)
        self.events = sorted(((int(r), SIM_EVENT.get(k, k), int(v)) for r, k, v in events),
                             key=lambda e: e[0])
        blob, off = pack_strings(names)
        self._blob = ctypes.create_string_buffer(blob, len(blob) + 1)
        self._off = off
        inc0 = np.ascontiguousarray(inc0, dtype=np.int64)
        dead = np.ascontiguousarray(dead, dtype=np.uint8)
        prev = os.environ.get("ORC_SIM_THREADS")
        if threads:
            os.environ["ORC_SIM_THREADS"] = str(int(threads))
        try:
            self.h = lib().orc_sim_new(self.N, seed, susp_rounds, now0, self._blob, off.ctypes.data,
                                       inc0.ctypes.data, dead.ctypes.data)
        finally:
            if threads:
                if prev is None:
                    os.environ.pop("ORC_SIM_THREADS", None)
                else:
                    os.environ["ORC_SIM_THREADS"] = prev

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_sim_free(self.h)
            self.h = None

    def step(self):
        r = self.round
        for er, k, v in self.events:
            if er == r:
                lib().orc_sim_event(self.h, k, v)
        lib().orc_sim_step(self.h)

    @property
    def round(self):
        return lib().orc_sim_round(self.h)

    def checksums(self):
        out = np.empty(self.N, dtype=np.uint32)
        lib().orc_sim_checksums(self.h, out.ctypes.data)
        return out

    def view(self, v):
        st = np.empty(self.N, dtype=np.uint8)
        inc = np.empty(self.N, dtype=np.int64)
        lib().orc_sim_view(self.h, v, st.ctypes.data, inc.ctypes.data)
        return st, inc

    def converged(self):
        return bool(lib().orc_sim_converged(self.h))

    def piggyback(self):
        out = np.empty(self.N, dtype=np.uint32)
        lib().orc_sim_piggyback(self.h, out.ctypes.data)
        return out

    def stats(self):
        out = np.zeros(4, dtype=np.uint64)
        lib().orc_sim_stats(self.h, out.ctypes.data)
        return dict(zip(["pings", "pingreqs", "fullsyncs", "applied"], (int(x) for x in out)))


class DampCfg(ctypes.Structure):
    """orc_damp_cfg (config.js:60-71 damp fields)."""
    _fields_ = [("enabled", ctypes.c_int), ("initial", ctypes.c_double), ("min", ctypes.c_double),
                ("max", ctypes.c_double), ("penalty", ctypes.c_double), ("suppress_limit", ctypes.c_double),
                ("half_life", ctypes.c_double)]


DAMP_DEFAULTS = {"dampScoringEnabled": True, "dampScoringInitial": 0, "dampScoringMin": 0, "dampScoringMax": 10000,
                 "dampScoringPenalty": 500, "dampScoringSuppressLimit": 5000, "dampScoringHalfLife": 60}


def damp_cfg(config=None):
    """A DampCfg from reference config keys (missing keys take config.js's defaults)."""
    c = dict(DAMP_DEFAULTS, **(config or {}))
    return DampCfg(int(bool(c["dampScoringEnabled"])), c["dampScoringInitial"], c["dampScoringMin"],
                   c["dampScoringMax"], c["dampScoringPenalty"], c["dampScoringSuppressLimit"],
                   c["dampScoringHalfLife"])


def js_pow(x, y):
    return lib().orc_js_pow(x, y)


def js_round(x):
    return lib().orc_js_round(x)


def damp_decayed(cfg, last_score, last_ts, now):
    return lib().orc_damp_decayed(ctypes.byref(cfg), last_score, int(last_ts), int(now))


def damp_penalized(cfg, last_score, last_ts, now):
    e = ctypes.c_int()
    s = lib().orc_damp_penalized(ctypes.byref(cfg), last_score, int(last_ts), int(now), ctypes.byref(e))
    return s, bool(e.value)


def damp_decay_all(cfg, exists, last_score, last_ts, now, score):
    """In place over numpy arrays (u8, f64, i64, f64)."""
    lib().orc_damp_decay_all(ctypes.byref(cfg), exists.ctypes.data, last_score.ctypes.data, last_ts.ctypes.data,
                             len(exists), int(now), score.ctypes.data)
