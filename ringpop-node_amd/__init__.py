"""ringpop-node_amd — Python host mirror of ringpop-node's hot-path API over librpamd.so.

The compute lives in HIP kernels behind the C ABI in include/ringpop_amd.h; this module is a
thin ctypes binding plus a `HashRing` class that keeps the reference's method names,
argument meanings and error behaviour (lib/ring/index.js), so parity tests read like the
reference's own tests (test/unit/ring-test.js, hashring_test.js). The Node N-API binding of
the same C ABI lives in js/ (the drop-in for lib/ring).

There is no CPU fallback: if librpamd.so is missing or no HIP device is visible, calls that
need the GPU raise RingpopAmdError.

The directory name contains a hyphen, so import it by path:
    spec = importlib.util.spec_from_file_location("ringpop_node_amd", ".../ringpop-node_amd/__init__.py")
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RP_AMD_LIB") or os.path.join(_HERE, "librpamd.so")  # override: A/B builds
NULL_ID = 0xFFFFFFFF

_lib = None


class RingpopAmdError(RuntimeError):
    pass


def build(arch="gfx950", jobs=8):
    """Compile librpamd.so in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-j%d" % jobs, "-C", os.path.join(_HERE, "csrc"), "ARCH=" + arch])


# name -> (restype, argtypes); every symbol declared in include/ringpop_amd.h
_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I32 = ctypes.c_int32
_INT = ctypes.c_int
SIGNATURES = {
    "rp_last_error": (ctypes.c_char_p, []),
    "rp_version": (_U32, []),
    "rp_device_count": (_INT, [_P]),
    "rp_hash32": (_U32, [ctypes.c_char_p, ctypes.c_size_t]),
    "rp_hash32_batch_dev": (_INT, [_P, _P, _U64, _P, _P]),
    "rp_hash32_long_dev": (_INT, [_P, _U64, _P, _P]),
    "rp_hash32_long_multi_dev": (_INT, [_P, _U64, _U32, _P, _P]),
    "rp_gen_uuid_keys_dev": (_INT, [_U32, _U64, _U64, _P, _P]),
    "rp_ring_create": (_INT, [_U32, _INT, _P]),
    "rp_ring_destroy": (_INT, [_P]),
    "rp_ring_add_remove": (_INT, [_P, _P, _P, _U32, _P, _P, _P, _U32, _P, _P]),
    "rp_ring_checksum": (_INT, [_P, _P, _P]),
    "rp_ring_checksum_string": (_INT, [_P, _P, _U64, _P]),
    "rp_ring_server_count": (_INT, [_P, _P]),
    "rp_ring_token_count": (_INT, [_P, _P]),
    "rp_ring_has_server": (_INT, [_P, _P, _U32, _P]),
    "rp_ring_server_id": (_INT, [_P, _P, _U32, _P]),
    "rp_ring_owner_name": (_P, [_P, _U32, _P]),
    "rp_ring_servers": (_INT, [_P, _P, _U32, _P]),
    "rp_ring_dump": (_INT, [_P, _P, _P, _U32]),
    "rp_ring_lookup": (_INT, [_P, _P, _P, _U32, _U64, _P]),
    "rp_ring_lookupn": (_INT, [_P, _P, _P, _U32, _U64, _I32, _P, _P]),
    "rp_ring_lookup_hashes": (_INT, [_P, _P, _U64, _P]),
    "rp_ring_lookupn_hashes": (_INT, [_P, _P, _U64, _I32, _P, _P]),
    "rp_ring_lookup_dev": (_INT, [_P, _P, _P, _U32, _U64, _P, _P]),
    "rp_ring_lookupn_dev": (_INT, [_P, _P, _P, _U32, _U64, _I32, _P, _P, _P]),
    "rp_ring_lookupn_hashes_dev": (_INT, [_P, _P, _U64, _I32, _P, _P, _P]),
    "rp_ring_group_keys_dev": (_INT, [_P, _P, _P, _U32, _U64, _U32, _P, _P, _P, _P, _P]),
    "rp_ring_group_keys": (_INT, [_P, _P, _P, _U32, _U64, _U32, _P, _P, _P, _P]),
    "rp_ring_group_hashes": (_INT, [_P, _P, _U64, _U32, _P, _P, _P, _P]),
    "rp_members_create": (_INT, [_U32, _INT, _P]),
    "rp_members_destroy": (_INT, [_P]),
    "rp_members_intern": (_INT, [_P, _P, _P, _U32, _P]),
    "rp_members_set_local": (_INT, [_P, _U32]),
    "rp_members_update": (_INT, [_P, _P, _P, _P, _U32, ctypes.c_int64, _P, _P, _P, _P]),
    "rp_members_update_dev": (_INT, [_P, _P, _P, _P, _U32, ctypes.c_int64, _P, _P, _P, _P, _P]),
    "rp_members_update_range_dev": (_INT, [_P, _P, _P, _P, _U32, ctypes.c_int64, _U32, _U32, _P, _P, _P, _P, _P]),
    "rp_members_rows_copy": (_INT, [_P, _P, _U32, _U32, ctypes.c_int, _P]),
    "rp_members_set": (_INT, [_P, _P, _P, _P, _U32, _P, _P]),
    "rp_members_set_dev": (_INT, [_P, _P, _P, _P, _U32, _P, _P, _P]),
    "rp_members_checksum": (_INT, [_P, _P, _P]),
    "rp_members_compute_checksum": (_INT, [_P]),
    "rp_members_checksum_string": (_INT, [_P, _P, _U64, _P]),
    "rp_members_dump": (_INT, [_P, _P, _P, _P, _U32]),
    "rp_members_count": (_INT, [_P, _P]),
    "rp_wire_encode_changes_dev": (_INT, [_P, _U32, _P, _U64, _P, _P, _P, _P, _P, _P, _INT, _INT, _P, _P, _P, _P,
                                          _P, _P]),
    "rp_wire_encode_changes": (_INT, [_P, _U32, _P, _P, _P, _P, _P, _P, _P, _INT, _INT, _P, _P, _P, _P, _U64, _P]),
    "rp_wire_decode_changes": (_INT, [_P, _P, _P, _U32, _P, _U32, _P, _P, _P, _P, _P, _P]),
    "rp_wire_decode_changes_dev": (_INT, [_P, _P, _P, _U32, _P, _U32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                          _P, _P]),
    "rp_sim_create": (_INT, [_U32, _P, _P, _P, _P, _U32, _U32, ctypes.c_int64, _INT, _P]),
    "rp_sim_destroy": (_INT, [_P]),
    "rp_sim_step": (_INT, [_P, _U32]),
    "rp_sim_step_async": (_INT, [_P, _U32]),
    "rp_sim_sync": (_INT, [_P]),
    "rp_sim_round": (_INT, [_P, _P]),
    "rp_sim_checksums": (_INT, [_P, _P]),
    "rp_sim_view": (_INT, [_P, _U32, _P, _P]),
    "rp_sim_converged": (_INT, [_P, _P]),
    "rp_sim_stats": (_INT, [_P, _P]),
    "rp_sim_create_shard": (_INT, [_U32, _P, _P, _P, _P, _U32, _U32, ctypes.c_int64, _INT, _P, _U32, _U32, _P]),
    "rp_sim_shard_info": (_INT, [_P, _P, _P, _P, _P]),
    "rp_sim_stage": (_INT, [_P, _INT]),
    "rp_sim_outbox": (_INT, [_P, _P, _P, _P]),
    "rp_sim_inbox": (_INT, [_P, _P, _P, _P]),
    "rp_sim_exchange_local": (_INT, [_P, _U32]),
    "rp_sim_wait_stream": (_INT, [_P, _P]),
    "rp_sim_order_stream": (_INT, [_P, _P]),
    "rp_sim_join_export": (_INT, [_P, _P, _P, _P]),
    "rp_sim_join_import": (_INT, [_P]),
    "rp_sim_join_exchange_local": (_INT, [_P, _U32]),
    "rp_sim_converged_local": (_INT, [_P, _P]),
    "rp_sim_create_scenario": (_INT, [_U32, _P, _P, _P, _P, _U32, _U32, ctypes.c_int64, _INT, _P, _U32, _U32, _P, _U32,
                                      _P]),
    "rp_sim_piggyback": (_INT, [_P, _P]),
    "rp_wire_encode_dev": (_INT, [_P, _U32, _P, _U64, _P, _INT, _INT, _P, _P, _P, _P]),
    "rp_wire_encode": (_INT, [_P, _U32, _P, _P, _INT, _INT, _P, _P, _U64, _P]),
    "rp_wire_decode_dev": (_INT, [_P, _P, _P, _U32, _P, _U32, _P, _P, _P, _P]),
    "rp_wire_decode": (_INT, [_P, _P, _P, _U32, _P, _U32, _P, _P, _P]),
    "rp_sim_counters": (_INT, [_P, _P]),
    "rp_members_defer_checksum": (_INT, [_P, _INT]),
    "rp_members_checksum_shard": (_INT, [_P, _U32, _U32, _U32]),
    "rp_members_checksum_history": (_INT, [_P, _P, _P, _U32, _P]),
    "rp_members_checksum_history_drain": (_INT, [_P, _U32]),
    "rp_ring_service": (_INT, [_P, _U32]),
    "rp_members_damp_configure": (_INT, [_P, _P]),
    "rp_members_damp_last": (_INT, [_P, _P, _P, _U32]),
    "rp_members_damp_decay": (_INT, [_P, ctypes.c_int64]),
    "rp_members_damp_decay_dev": (_INT, [_P, ctypes.c_int64, _P]),
    "rp_members_damp_dump": (_INT, [_P, _P, _P, _P, _U32]),
    "rp_copy": (_INT, [_P, _P, _U64, _P]),
}

STATUS = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}
STATUS_NAME = {v: k for k, v in STATUS.items()}


def lib():
    """Load librpamd.so (fails loudly; there is no fallback implementation)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RingpopAmdError("librpamd.so not built: run `make -C ringpop-node_amd/csrc` "
                                  "(or __graft_entry__.build())")
        # PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7). Loading torch
        # first makes librpamd bind to that same runtime instance, so device pointers and
        # streams from torch tensors are valid in our kernels (one HIP runtime per process).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _is_array_index(k):
    """A property name JS orders first in Object.keys: the canonical decimal of an integer in
    [0, 2^32 - 2]."""
    return k.isdigit() and k.isascii() and (k == "0" or k[0] != "0") and int(k) < 0xFFFFFFFF


def check(rc):
    if rc != 0:
        raise RingpopAmdError("librpamd: %s (status %d)" % (lib().rp_last_error().decode(errors="replace"), rc))


def device_count():
    n = ctypes.c_int()
    check(lib().rp_device_count(ctypes.byref(n)))
    return n.value


def hash32(s):
    """farmhash.hash32 (npm farmhash ^0.2.0) — host C++ farmhashmk::Hash32."""
    b = s.encode() if isinstance(s, str) else bytes(s)
    return lib().rp_hash32(b, len(b))


def _pack(strs):
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strs]
    off = np.zeros(len(bs) + 1, dtype=np.uint32)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs])
    blob = b"".join(bs)
    return ctypes.create_string_buffer(blob, len(blob) + 1), off


def _ptr(a):
    return None if a is None else a.ctypes.data


def gen_uuid_keys_dev(seed, k0, n, out_ptr, stream=None):
    """Fill a device buffer (>= 36*n bytes, 4-byte aligned) with the synthetic key stream."""
    check(lib().rp_gen_uuid_keys_dev(seed, k0, n, out_ptr, stream))


class HashRing:
    """Mirror of lib/ring/index.js HashRing (25-189) backed by the device ring.

    options: {'replicaPoints': int, 'hashFunc': callable(str)->uint32} as in the reference
    constructor (lib/ring/index.js:25-34). Events 'added', 'removed', 'checksumComputed'.
    """

    def __init__(self, options=None, device=0):
        self.options = dict(options or {})
        self.replicaPoints = self.options.get("replicaPoints") or 100
        self.hashFunc = self.options.get("hashFunc")  # None => device farmhash32
        self._listeners = {}
        h = ctypes.c_void_p()
        check(lib().rp_ring_create(self.replicaPoints, device, ctypes.byref(h)))
        self._h = h
        self._names = {}
        # servers (lib/ring/index.js:32): name -> True in insertion order (Object.keys order),
        # kept from the same add / remove decisions the device makes and checked against it
        self._servers = {}

    def close(self):
        if getattr(self, "_h", None):
            lib().rp_ring_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- events (EventEmitter subset)
    def on(self, ev, fn):
        self._listeners.setdefault(ev, []).append(fn)
        return self

    def emit(self, ev, *args):
        for fn in list(self._listeners.get(ev, [])):
            fn(*args)

    # -- mutation
    def _tokens(self, names):
        if self.hashFunc is None or not names:
            return None
        R = self.replicaPoints
        return np.array([self.hashFunc(s + str(i)) & 0xFFFFFFFF for s in names for i in range(R)],
                        dtype=np.uint32)

    def service(self, idle_ms):
        """rp_ring_service: idle_ms > 0 answers one-key lookup / lookupN calls through the resident
        lookup service (no launch per call); 0 turns it off."""
        check(lib().rp_ring_service(self._h, int(idle_ms)))

    def addRemoveServers(self, serversToAdd=None, serversToRemove=None):
        """lib/ring/index.js:60-94; returns ringChanged. The reference's per-name decisions (adds in
        order, then removes, each against the servers map) are made first; only the names that
        change go to the device, and the map is committed after the device call succeeded."""
        over = {}
        add, rem = [], []
        for a in serversToAdd or []:
            if not over.get(a, a in self._servers):
                over[a] = True
                add.append(a)
        for r in serversToRemove or []:
            if over.get(r, r in self._servers):
                over[r] = False
                rem.append(r)
        if not add and not rem:
            return False
        ab, ao = _pack(add)
        rb, ro = _pack(rem)
        at, rt = self._tokens(add), self._tokens(rem)  # kept alive across the call
        changed = ctypes.c_int()
        check(lib().rp_ring_add_remove(self._h, ab, ao.ctypes.data, len(add), _ptr(at),
                                       rb, ro.ctypes.data, len(rem), _ptr(rt), ctypes.byref(changed)))
        if not changed.value:
            raise RingpopAmdError("the device ring did not change for add %r remove %r" % (add, rem))
        for a in add:
            self._servers[a] = True
        for r in rem:
            del self._servers[r]
        self.emit("checksumComputed")
        return True

    def addServer(self, name):
        """lib/ring/index.js:39-48"""
        if self.hasServer(name):
            return
        self.addRemoveServers([name], None)
        self.emit("added", name)

    def removeServer(self, name):
        """lib/ring/index.js:124-133"""
        if not self.hasServer(name):
            return
        self.addRemoveServers(None, [name])
        self.emit("removed", name)

    # -- state
    @property
    def checksum(self):
        v, s = ctypes.c_uint32(), ctypes.c_int()
        check(lib().rp_ring_checksum(self._h, ctypes.byref(v), ctypes.byref(s)))
        if not s.value:
            return None
        if self.hashFunc is not None:
            return self.hashFunc(self.checksum_string()) & 0xFFFFFFFF
        return v.value

    def checksum_string(self):
        n = ctypes.c_uint64()
        check(lib().rp_ring_checksum_string(self._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        check(lib().rp_ring_checksum_string(self._h, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value].decode()

    def getServerCount(self):
        v = ctypes.c_uint32()
        check(lib().rp_ring_server_count(self._h, ctypes.byref(v)))
        return v.value

    @property
    def size(self):
        """rbtree.size"""
        v = ctypes.c_uint32()
        check(lib().rp_ring_token_count(self._h, ctypes.byref(v)))
        return v.value

    def hasServer(self, name):
        b = name.encode()
        v = ctypes.c_int()
        check(lib().rp_ring_has_server(self._h, b, len(b), ctypes.byref(v)))
        return bool(v.value)

    def server_ids(self):
        n = ctypes.c_uint32()
        check(lib().rp_ring_servers(self._h, None, 0, ctypes.byref(n)))
        out = np.empty(max(n.value, 1), dtype=np.uint32)
        check(lib().rp_ring_servers(self._h, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[:n.value]

    @property
    def servers(self):
        """lib/ring/index.js:32 (a copy)"""
        return dict(self._servers)

    def getStats(self):
        """lib/ring/index.js:111-116 (servers in Object.keys order: array-index names ascending,
        then the others in insertion order)"""
        idx = sorted((int(k), k) for k in self._servers if _is_array_index(k))
        return {"checksum": self.checksum,
                "servers": [k for _, k in idx] + [k for k in self._servers if not _is_array_index(k)]}

    def name(self, sid):
        sid = int(sid)
        if sid == NULL_ID:
            return None
        s = self._names.get(sid)
        if s is None:
            n = ctypes.c_uint32()
            p = lib().rp_ring_owner_name(self._h, sid, ctypes.byref(n))
            if not p:
                raise RingpopAmdError("unknown server id %d" % sid)
            s = ctypes.string_at(p, n.value).decode()
            self._names[sid] = s
        return s

    def server_id(self, name):
        b = name.encode()
        v = ctypes.c_uint32()
        check(lib().rp_ring_server_id(self._h, b, len(b), ctypes.byref(v)))
        return v.value

    def dump(self):
        m = self.size
        t = np.empty(max(m, 1), dtype=np.uint32)
        o = np.empty(max(m, 1), dtype=np.uint32)
        check(lib().rp_ring_dump(self._h, t.ctypes.data, o.ctypes.data, m))
        return t[:m], o[:m]

    # -- lookups (single-key reference API; batch forms below)
    def lookup(self, key):
        """lib/ring/index.js:145-154"""
        ids = self.lookup_ids([str(key)])
        return self.name(ids[0])

    def lookupN(self, key, n):
        """lib/ring/index.js:157-189"""
        ids, cnt = self.lookupn_ids([str(key)], n)
        return [self.name(x) for x in ids[0][:cnt[0]]]

    def _key_pack(self, keys):
        if isinstance(keys, np.ndarray) and keys.ndim == 2 and keys.dtype == np.uint8:
            return np.ascontiguousarray(keys), None, keys.shape[1], keys.shape[0]
        bs = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        if bs:
            off[1:] = np.cumsum([len(b) for b in bs])
        blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
        return blob, off, 0, len(bs)

    def lookup_ids(self, keys):
        """Batched lookup: owner ids (NULL_ID = null)."""
        if self.hashFunc is not None:
            hs = np.array([self.hashFunc(k) & 0xFFFFFFFF for k in keys], dtype=np.uint32)
            return self.lookup_hashes(hs)
        blob, off, stride, n = self._key_pack(keys)
        out = np.empty(max(n, 1), dtype=np.uint32)
        check(lib().rp_ring_lookup(self._h, blob.ctypes.data, _ptr(off), stride, n, out.ctypes.data))
        return out[:n]

    def lookupn_ids(self, keys, n):
        """Batched lookupN: (owners[k, max(n,1)], counts[k])."""
        if self.hashFunc is not None:
            hs = np.array([self.hashFunc(k) & 0xFFFFFFFF for k in keys], dtype=np.uint32)
            return self.lookupn_hashes(hs, n)
        blob, off, stride, k = self._key_pack(keys)
        w = max(int(n), 1)
        out = np.empty((max(k, 1), w), dtype=np.uint32)
        cnt = np.empty(max(k, 1), dtype=np.uint8)
        check(lib().rp_ring_lookupn(self._h, blob.ctypes.data, _ptr(off), stride, k, int(n), out.ctypes.data,
                                    cnt.ctypes.data))
        return out[:k], cnt[:k]

    def lookup_hashes(self, hashes):
        hs = np.ascontiguousarray(hashes, dtype=np.uint32)
        out = np.empty(max(len(hs), 1), dtype=np.uint32)
        check(lib().rp_ring_lookup_hashes(self._h, hs.ctypes.data, len(hs), out.ctypes.data))
        return out[:len(hs)]

    def lookupn_hashes(self, hashes, n):
        hs = np.ascontiguousarray(hashes, dtype=np.uint32)
        w = max(int(n), 1)
        out = np.empty((max(len(hs), 1), w), dtype=np.uint32)
        cnt = np.empty(max(len(hs), 1), dtype=np.uint8)
        check(lib().rp_ring_lookupn_hashes(self._h, hs.ctypes.data, len(hs), int(n), out.ctypes.data,
                                           cnt.ctypes.data))
        return out[:len(hs)], cnt[:len(hs)]

    # -- keys grouped by owner: handleOrProxyAll (index.js:609-667) / lookupKeys (send.js:171-179)
    def group_ids(self, keys, self_id=NULL_ID):
        """(dests, group_off, perm): owners in first-seen order, group bounds, key indices."""
        n = len(keys)
        dests = np.empty(max(n, 1), dtype=np.uint32)
        goff = np.empty(max(n, 1) + 1, dtype=np.uint32)
        perm = np.empty(max(n, 1), dtype=np.uint32)
        nd = ctypes.c_uint32()
        if self.hashFunc is not None:
            hs = np.array([self.hashFunc(k) & 0xFFFFFFFF for k in keys], dtype=np.uint32)
            check(lib().rp_ring_group_hashes(self._h, hs.ctypes.data, n, self_id, dests.ctypes.data,
                                             goff.ctypes.data, perm.ctypes.data, ctypes.byref(nd)))
        else:
            blob, off, stride, n = self._key_pack(keys)
            check(lib().rp_ring_group_keys(self._h, blob.ctypes.data, _ptr(off), stride, n, self_id,
                                           dests.ctypes.data, goff.ctypes.data, perm.ctypes.data, ctypes.byref(nd)))
        k = nd.value
        return dests[:k], goff[:k + 1], perm[:n]

    def groupBy(self, keys, whoami=None):
        """_.groupBy(keys, ringpop.lookup) as handleOrProxyAll builds keysByDest (index.js:616):
        {dest: [keys in input order]} with dests in first-seen order; an empty ring's null
        owner falls back to whoami (RingPop.lookup, index.js:434-451)."""
        keys = [k if isinstance(k, (bytes, np.ndarray)) else str(k) for k in keys]
        dests, goff, perm = self.group_ids(keys, self_id=NULL_ID)
        out = {}
        for g, d in enumerate(dests):
            out[whoami if d == NULL_ID else self.name(d)] = [keys[i] for i in perm[goff[g]:goff[g + 1]]]
        return out

    def lookupKeys(self, keys, whoami=None):
        """RequestProxySend.lookupKeys (lib/request-proxy/send.js:171-179)."""
        dests, _, _ = self.group_ids([str(k) for k in keys], self_id=NULL_ID)
        return [whoami if d == NULL_ID else self.name(d) for d in dests]

    def group_dev(self, keys_ptr, n, dests_ptr, goff_ptr, perm_ptr, ndest_ptr, self_id=NULL_ID, stride=36,
                  off_ptr=None, stream=None):
        check(lib().rp_ring_group_keys_dev(self._h, keys_ptr, off_ptr, stride, n, self_id, dests_ptr, goff_ptr,
                                           perm_ptr, ndest_ptr, stream))

    # -- device-resident hot path (pointers from torch tensors / hipMalloc)
    def lookupn_dev(self, keys_ptr, n, nrep, owners_ptr, counts_ptr=None, stride=36, off_ptr=None, stream=None):
        check(lib().rp_ring_lookupn_dev(self._h, keys_ptr, off_ptr, stride, n, nrep, owners_ptr, counts_ptr, stream))

    def lookup_dev(self, keys_ptr, n, owners_ptr, stride=36, off_ptr=None, stream=None):
        check(lib().rp_ring_lookup_dev(self._h, keys_ptr, off_ptr, stride, n, owners_ptr, stream))


class DampConfig(ctypes.Structure):
    """rp_damp_config (include/ringpop_amd.h)."""
    _fields_ = [("enabled", ctypes.c_int), ("initial", ctypes.c_double), ("min", ctypes.c_double),
                ("max", ctypes.c_double), ("penalty", ctypes.c_double), ("suppress_limit", ctypes.c_double),
                ("half_life", ctypes.c_double)]


DAMP_DEFAULTS = {"dampScoringEnabled": True, "dampScoringInitial": 0, "dampScoringMin": 0, "dampScoringMax": 10000,
                 "dampScoringPenalty": 500, "dampScoringSuppressLimit": 5000, "dampScoringHalfLife": 60}


class Membership:
    """Device member table behind Membership.update / computeChecksum
    (lib/membership/index.js:48-123, 249-324; rules: lib/membership/member.js:71-202).

    Addresses are interned to ids; `update` takes the reference's change dicts
    ({address, status, incarnationNumber}) or id/status/inc arrays (`update_ids`).
    """

    def __init__(self, whoami=None, capacity=1024, device=0, now=None):
        h = ctypes.c_void_p()
        check(lib().rp_members_create(capacity, device, ctypes.byref(h)))
        self._h = h
        self._names = []
        self._ids = {}
        self.now = now or (lambda: 0)
        # isReady + the stash of remote changes received before it (index.js:259-265), kept on
        # the host as the reference's JS side keeps it; set() merges it on the device
        self.is_ready = True
        self._stash = []
        self._stash_nulled = False
        if whoami is not None:
            check(lib().rp_members_set_local(self._h, self.intern([whoami])[0]))

    def close(self):
        if getattr(self, "_h", None):
            lib().rp_members_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def intern(self, addresses):
        new = [a for a in dict.fromkeys(addresses) if a not in self._ids]
        if new:
            buf, off = _pack(new)
            ids = np.empty(len(new), dtype=np.uint32)
            check(lib().rp_members_intern(self._h, buf, off.ctypes.data, len(new), ids.ctypes.data))
            for a, i in zip(new, ids):
                self._ids[a] = int(i)
                while len(self._names) <= i:
                    self._names.append(None)
                self._names[int(i)] = a
        return [self._ids[a] for a in addresses]

    def address(self, i):
        return self._names[i]

    def set_ready(self, ready):
        self.is_ready = bool(ready)

    def update_ids(self, ids, status, inc, now_ms=None, is_local=False):
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        st = np.ascontiguousarray(status, dtype=np.uint8)
        inc = np.ascontiguousarray(inc, dtype=np.int64)
        k = len(ids)
        if not is_local and not self.is_ready:  # stashed, nothing applied (index.js:259-265)
            if not self._stash_nulled:
                self._stash.append((ids.copy(), st.copy(), inc.copy()))
            z = np.zeros(k, dtype=np.uint8)
            return z, st.copy(), inc.copy(), 0
        app = np.empty(max(k, 1), dtype=np.uint8)
        nst = np.empty(max(k, 1), dtype=np.uint8)
        ninc = np.empty(max(k, 1), dtype=np.int64)
        na = ctypes.c_uint32()
        now_ms = self.now() if now_ms is None else now_ms
        check(lib().rp_members_update(self._h, ids.ctypes.data, st.ctypes.data, inc.ctypes.data, k, int(now_ms),
                                      app.ctypes.data, nst.ctypes.data, ninc.ctypes.data, ctypes.byref(na)))
        return app[:k], nst[:k], ninc[:k], na.value

    def update(self, changes, now_ms=None):
        """Membership.update(changes): returns the applied updates (dicts) in batch order."""
        changes = changes if isinstance(changes, list) else [changes]
        ids = self.intern([c["address"] for c in changes])
        app, nst, ninc, _ = self.update_ids(ids, [STATUS[c["status"]] for c in changes],
                                            [c["incarnationNumber"] for c in changes], now_ms)
        out = []
        for c, a, s_, i_ in zip(changes, app, nst, ninc):
            if a:
                u = dict(c)
                u["status"] = STATUS_NAME[int(s_)]
                u["incarnationNumber"] = int(i_)
                out.append(u)
        return out

    def set(self):
        """Membership.set (index.js:208-247): merge the stash on the device
        (mergeMembershipChangesets) and set the picked members; returns the picked changes'
        (address, status, inc) in first-seen order."""
        if self.is_ready or self._stash_nulled or not self._stash:
            return []
        ids = np.concatenate([x[0] for x in self._stash])
        st = np.concatenate([x[1] for x in self._stash])
        inc = np.concatenate([x[2] for x in self._stash])
        pick = np.empty(len(ids), dtype=np.uint32)
        npick = ctypes.c_uint32()
        check(lib().rp_members_set(self._h, ids.ctypes.data, st.ctypes.data, inc.ctypes.data, len(ids),
                                   pick.ctypes.data, ctypes.byref(npick)))
        self._stash = []
        self._stash_nulled = True
        return [(self._names[int(ids[j])], STATUS_NAME[int(st[j])], int(inc[j])) for j in pick[:npick.value]]

    @property
    def checksum(self):
        v, s_ = ctypes.c_uint32(), ctypes.c_int()
        check(lib().rp_members_checksum(self._h, ctypes.byref(v), ctypes.byref(s_)))
        return v.value if s_.value else None

    def compute_checksum(self):
        check(lib().rp_members_compute_checksum(self._h))
        return self.checksum

    def generate_checksum_string(self):
        n = ctypes.c_uint64()
        check(lib().rp_members_checksum_string(self._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        check(lib().rp_members_checksum_string(self._h, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value].decode()

    def dump(self):
        n = ctypes.c_uint32()
        check(lib().rp_members_count(self._h, ctypes.byref(n)))
        m = n.value
        ex = np.empty(max(m, 1), dtype=np.uint8)
        st = np.empty(max(m, 1), dtype=np.uint8)
        inc = np.empty(max(m, 1), dtype=np.int64)
        check(lib().rp_members_dump(self._h, ex.ctypes.data, st.ctypes.data, inc.ctypes.data, m))
        return ex[:m], st[:m], inc[:m]

    def member(self, address):
        i = self._ids.get(address)
        if i is None:
            return None
        ex, st, inc = self.dump()
        if not ex[i]:
            return None
        return {"address": address, "status": STATUS_NAME[int(st[i])], "incarnationNumber": int(inc[i])}

    def update_dev(self, d_ids, d_status, d_inc, k, now_ms, d_applied=None, d_new_status=None, d_new_inc=None,
                   d_n_applied=None, stream=None):
        check(lib().rp_members_update_dev(self._h, d_ids, d_status, d_inc, k, int(now_ms), d_applied, d_new_status,
                                          d_new_inc, d_n_applied, stream))

    def update_range_dev(self, d_ids, d_status, d_inc, k, now_ms, id_lo, id_hi, d_applied=None, d_new_status=None,
                         d_new_inc=None, d_n_applied=None, stream=None):
        """update_dev applied only to the changes whose id lies in [id_lo, id_hi) (whole buckets of
        4,096 ids; rp_members_update_range_dev): no checksum, other changes' outputs untouched."""
        check(lib().rp_members_update_range_dev(self._h, d_ids, d_status, d_inc, k, int(now_ms), id_lo, id_hi,
                                                d_applied, d_new_status, d_new_inc, d_n_applied, stream))

    def rows_copy(self, d_buf, id_lo, id_hi, into_table, stream=None):
        """Member rows [id_lo, id_hi) (8 B each) to (into_table False) or from a device buffer."""
        check(lib().rp_members_rows_copy(self._h, d_buf, id_lo, id_hi, 1 if into_table else 0, stream))

    def checksum_shard(self, nshards, shard, history_cap=0):
        """From now on checksum only update batches b % nshards == shard (rp_members_checksum_shard),
        recording each one's checksum when history_cap > 0."""
        check(lib().rp_members_checksum_shard(self._h, nshards, shard, history_cap))

    def checksum_history(self):
        """This handle's recorded per-batch checksums: (hash uint32[], applied uint8[])."""
        n = ctypes.c_uint32()
        check(lib().rp_members_checksum_history(self._h, None, None, 0, ctypes.byref(n)))
        h = np.empty(max(n.value, 1), dtype=np.uint32)
        a = np.empty(max(n.value, 1), dtype=np.uint8)
        check(lib().rp_members_checksum_history(self._h, h.ctypes.data, a.ctypes.data, n.value, ctypes.byref(n)))
        return h[:n.value], a[:n.value]

    # ---- flap-damping scores (member.js:45-66,133-153; index.js:330-383) ----
    def damp_configure(self, config=None):
        """Track dampScore on the device with the reference's config keys (config.js:60-71;
        missing keys take its defaults)."""
        c = dict(DAMP_DEFAULTS, **(config or {}))
        cfg = DampConfig(int(bool(c["dampScoringEnabled"])), c["dampScoringInitial"], c["dampScoringMin"],
                         c["dampScoringMax"], c["dampScoringPenalty"], c["dampScoringSuppressLimit"],
                         c["dampScoringHalfLife"])
        check(lib().rp_members_damp_configure(self._h, ctypes.byref(cfg)))

    def damp_last(self, k):
        """(score after each change, suppressLimitExceeded flags) of the last update batch of k changes."""
        sc = np.empty(max(k, 1), dtype=np.float64)
        ex = np.empty(max(k, 1), dtype=np.uint8)
        check(lib().rp_members_damp_last(self._h, sc.ctypes.data, ex.ctypes.data, k))
        return sc[:k], ex[:k]

    def damp_decay(self, now_ms=None):
        """Membership._decayMembersDampScore at Date.now() = now_ms."""
        check(lib().rp_members_damp_decay(self._h, int(self.now() if now_ms is None else now_ms)))

    def damp_decay_dev(self, now_ms, stream=None):
        check(lib().rp_members_damp_decay_dev(self._h, int(now_ms), stream))

    def damp_dump(self):
        """Per id: dampScore, lastUpdateDampScore, lastUpdateTimestamp (0 = null)."""
        n = ctypes.c_uint32()
        check(lib().rp_members_count(self._h, ctypes.byref(n)))
        m = n.value
        sc = np.empty(max(m, 1), dtype=np.float64)
        ls = np.empty(max(m, 1), dtype=np.float64)
        ts = np.empty(max(m, 1), dtype=np.int64)
        check(lib().rp_members_damp_dump(self._h, sc.ctypes.data, ls.ctypes.data, ts.ctypes.data, m))
        return sc[:m], ls[:m], ts[:m]


class DistMembership(Membership):
    """Membership.update over G GPUs (membership merge): one replica of the member
    table per rank (one process per GPU). Every rank folds every batch (the fold is cheap and
    keeps each replica whole: any rank answers member reads); the per-batch checksums, whose
    string build and serial farmhash chain are most of a batch (index.js:48-75, 306-309), are
    divided among the ranks: rank g computes those of batches b with b % G == g. No per-batch
    collective: `checksums()` gathers the recorded per-batch values once (one all-gather).

    The batch stream must be the same on every rank (as the reference's is the same for one
    process). The device records at most `history_cap` of this rank's batches between two
    `checksums()` calls (an update past that fails with nothing applied); `checksums()` moves the
    record to the host and drains it, so a long-running replica keeps going."""

    def __init__(self, whoami=None, capacity=1024, device=0, history_cap=1 << 16, group=None):
        import torch.distributed as dist
        super().__init__(whoami=whoami, capacity=capacity, device=device)
        self._dist = dist
        self._group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # the gathered record (round 5): values interleaved so far and the carried
        # value; each gather moves only the entries recorded since the previous one
        self._out = []
        self._cur = None
        self.checksum_shard(self.world, self.rank, history_cap)

    @property
    def checksum(self):
        """Membership.checksum after the last batch. With G = 1 the device's own value. With
        G > 1 the latest value lives on one rank, so reading it is a collective: use
        latest_checksum() on every rank (local_checksum() for this rank's own latest value)."""
        if self.world == 1:
            return Membership.checksum.fget(self)
        raise RingpopAmdError("DistMembership.checksum over %d ranks is a collective: call "
                              "latest_checksum() on every rank" % self.world)

    def local_checksum(self):
        """The checksum of the latest batch this rank hashed (b % G == rank), after its pending
        chains finish; no collective."""
        return Membership.checksum.fget(self)

    def latest_checksum(self):
        """Membership.checksum after the last batch (a collective: every rank calls it)."""
        self._gather()
        return self._cur

    def compute_checksum(self):
        """computeChecksum() of this rank's replica, which is the whole table: local, no collective."""
        check(lib().rp_members_compute_checksum(self._h))
        return Membership.checksum.fget(self)

    def _gather(self):
        """Drain this rank's device record, gather every rank's entries recorded since the last
        gather (one all-gather of the counts, one of the entries) and interleave them in batch
        order onto the host record."""
        import torch
        h, a = self.checksum_history()
        if len(h):
            check(lib().rp_members_checksum_history_drain(self._h, len(h)))
        if self.world > 1:
            # nccl (RCCL) gathers device tensors; gloo host tensors
            dev = "cuda" if self._dist.get_backend(self._group) == "nccl" else "cpu"
            n = torch.tensor([len(h)], dtype=torch.int64, device=dev)
            ns = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(self.world)]
            self._dist.all_gather(ns, n, group=self._group)
            ns = [int(x.item()) for x in ns]
            cap = max(ns)
            if cap == 0:
                return
            mine = torch.zeros(cap, 2, dtype=torch.int64)
            mine[:len(h), 0] = torch.from_numpy(h.astype(np.int64))
            mine[:len(h), 1] = torch.from_numpy(a.astype(np.int64))
            parts = [torch.zeros(cap, 2, dtype=torch.int64, device=dev) for _ in range(self.world)]
            self._dist.all_gather(parts, mine.to(dev), group=self._group)
            parts = [x.cpu().numpy() for x in parts]
        else:
            ns = [len(h)]
            parts = [np.stack([h.astype(np.int64), a.astype(np.int64)], axis=1)]
        ptr = [0] * self.world
        b0 = len(self._out)
        for b in range(b0, b0 + sum(ns)):
            g = b % self.world
            hv, av = parts[g][ptr[g]]
            ptr[g] += 1
            if av:
                self._cur = int(hv)
            self._out.append(self._cur)

    def checksums(self):
        """The checksum after every update batch since construction (None before the first
        applied one), in batch order: every rank's recorded values gathered and interleaved, a
        batch that applied nothing carrying the previous value forward (index.js:306-309).
        A collective: every rank calls it."""
        self._gather()
        return list(self._out)


class PartMembership(Membership):
    """Membership.update over G GPUs partitioned by member id (SURVEY §8e's row partition of
    lib/membership/index.js:249-324): rank g owns the ids [lo_g, hi_g) (equal runs of whole
    4,096-id buckets of the capacity given here; the last rank's run is open-ended), folds only
    the changes of its ids out of each batch (rp_members_update_range_dev) and keeps only its own
    rows current. The batch is on every rank (as the reference's one process holds it), so no
    change crosses ranks; every rank scans the batch and folds 1/G of it. The checksum hashes
    every row in address order, so compute_checksum() / dump() first bring the ranges together
    (one all-gather of 8 B per member: RCCL device tensors, or gloo host tensors) and are
    collectives. Per-change outputs (applied, new status / incarnation) are written on the rank
    that owns the change's id; update_dev returns nothing else. The replicated form
    (DistMembership) is what C3's per-batch checksums want; this one is for large batches whose
    fold is the cost."""

    BUCKET = 4096

    def __init__(self, whoami=None, capacity=1024, device=0, group=None):
        import torch.distributed as dist
        super().__init__(whoami=whoami, capacity=capacity, device=device)
        self._dist = dist
        self._group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.per_ids, self.id_lo, self.id_hi = self.partition(capacity, self.world, self.rank)

    @classmethod
    def partition(cls, capacity, world, rank):
        """(ids per rank, id_lo, id_hi) of rank's run: equal runs of whole buckets of the capacity,
        the last rank's run open-ended (0xFFFFF000, a bucket multiple past any table)."""
        nb = -(-max(int(capacity), 1) // cls.BUCKET)
        per = -(-nb // world) * cls.BUCKET
        lo = min(rank * per, nb * cls.BUCKET)
        hi = 0xFFFFF000 if rank == world - 1 else min((rank + 1) * per, nb * cls.BUCKET)
        return per, lo, hi

    def update_dev(self, d_ids, d_status, d_inc, k, now_ms, d_applied=None, d_new_status=None, d_new_inc=None,
                   d_n_applied=None, stream=None):
        """This rank's part of Membership.update over device buffers (stream-ordered, no sync)."""
        self.update_range_dev(d_ids, d_status, d_inc, k, now_ms, self.id_lo, self.id_hi, d_applied, d_new_status,
                              d_new_inc, d_n_applied, stream)

    def gather_rows(self):
        """Make this rank's table whole: every rank's own rows all-gathered (a collective)."""
        import torch
        n = ctypes.c_uint32()
        check(lib().rp_members_count(self._h, ctypes.byref(n)))
        nid = n.value
        if self.world == 1 or nid == 0:
            return
        per = self.per_ids
        if nid > self.world * per:
            raise RingpopAmdError("PartMembership: %d members outgrew the partition of %d ids; construct it "
                                  "with the capacity the table will reach" % (nid, self.world * per))
        lo, hi = min(self.id_lo, nid), min(self.rank * per + per, nid)
        sp = torch.cuda.current_stream().cuda_stream
        mine = torch.zeros(per * 8, dtype=torch.uint8, device="cuda")
        if hi > lo:
            self.rows_copy(mine.data_ptr(), lo, hi, False, sp)
        if self._dist.get_backend(self._group) == "nccl":
            full = torch.empty(self.world * per * 8, dtype=torch.uint8, device="cuda")
            self._dist.all_gather_into_tensor(full, mine, group=self._group)
        else:  # gloo: host tensors
            parts = [torch.empty(per * 8, dtype=torch.uint8) for _ in range(self.world)]
            self._dist.all_gather(parts, mine.cpu(), group=self._group)
            full = torch.cat(parts).cuda()
        for g in range(self.world):
            a, b = g * per, min(g * per + per, nid)
            if g != self.rank and b > a:
                self.rows_copy(full.data_ptr() + a * 8, a, b, True, sp)
        torch.cuda.current_stream().synchronize()

    @property
    def checksum(self):
        if self.world == 1:
            return Membership.checksum.fget(self)
        raise RingpopAmdError("PartMembership.checksum over %d ranks needs the rows together: call "
                              "compute_checksum() on every rank" % self.world)

    def compute_checksum(self):
        """computeChecksum() over the whole table (a collective: gathers the rows first)."""
        self.gather_rows()
        check(lib().rp_members_compute_checksum(self._h))
        return Membership.checksum.fget(self)

    def dump(self):
        """The whole table (a collective: gathers the rows first)."""
        self.gather_rows()
        return Membership.dump(self)


SIM_EVENT = {"kill": 0, "revive": 1, "leave": 2, "join": 3}


def _events(events):
    """(round, kind, node) triples -> rp_sim_event[] (uint32 x 4 each); kind a SIM_EVENT name or code."""
    ev = np.zeros((max(len(events), 1), 4), dtype=np.uint32)
    for i, (r, k, v) in enumerate(events):
        ev[i, :3] = (int(r), SIM_EVENT.get(k, k), int(v))
    return ev, len(events)


def _sim_create(names, inc0, dead, seed, suspicion_rounds, now0, device, bounds, nshards, shard, events):
    buf, off = _pack(names)
    inc0 = np.ascontiguousarray(inc0, dtype=np.int64)
    dead = np.ascontiguousarray(dead, dtype=np.uint8)
    if now0 is None:
        now0 = 1434401518824 + 10 ** 9
    ev, nev = _events(events or [])
    h = ctypes.c_void_p()
    check(lib().rp_sim_create_scenario(len(names), buf, off.ctypes.data, inc0.ctypes.data, dead.ctypes.data, seed,
                                       suspicion_rounds, int(now0), device,
                                       None if bounds is None else bounds.ctypes.data, nshards, shard,
                                       ev.ctypes.data, nev, ctypes.byref(h)))
    return h


class GossipSim:
    """N full ringpop nodes advanced in the deterministic gossip round model on the device
    (DESIGN.md §SWIM round model; oracle/orc_sim.c restates it on the CPU). events: scenario
    (round, kind, node) triples, kind in SIM_EVENT (include/ringpop_amd.h "Scenarios")."""

    def __init__(self, names, inc0, dead, seed=11, suspicion_rounds=25, now0=None, device=0, events=()):
        self.N = len(names)
        self._h = _sim_create(names, inc0, dead, seed, suspicion_rounds, now0, device, None, 1, 0, events)

    def close(self):
        if getattr(self, "_h", None):
            lib().rp_sim_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def step(self, rounds=1):
        check(lib().rp_sim_step(self._h, rounds))

    def step_async(self, rounds=1):
        check(lib().rp_sim_step_async(self._h, rounds))

    def sync(self):
        check(lib().rp_sim_sync(self._h))

    @property
    def round(self):
        v = ctypes.c_int64()
        check(lib().rp_sim_round(self._h, ctypes.byref(v)))
        return v.value

    def checksums(self):
        out = np.empty(self.N, dtype=np.uint32)
        check(lib().rp_sim_checksums(self._h, out.ctypes.data))
        return out

    def view(self, v):
        st = np.empty(self.N, dtype=np.uint8)
        inc = np.empty(self.N, dtype=np.int64)
        check(lib().rp_sim_view(self._h, v, st.ctypes.data, inc.ctypes.data))
        return st, inc

    def converged(self):
        v = ctypes.c_int()
        check(lib().rp_sim_converged(self._h, ctypes.byref(v)))
        return bool(v.value)

    def stats(self):
        out = np.zeros(4, dtype=np.uint64)
        check(lib().rp_sim_stats(self._h, out.ctypes.data))
        return dict(zip(["pings", "pingreqs", "fullsyncs", "applied"], (int(x) for x in out)))

    def piggyback(self):
        """Every node's dissemination.maxPiggybackCount."""
        out = np.empty(self.N, dtype=np.uint32)
        check(lib().rp_sim_piggyback(self._h, out.ctypes.data))
        return out

    def counters(self):
        out = np.zeros(8, dtype=np.uint64)
        check(lib().rp_sim_counters(self._h, out.ctypes.data))
        return dict(zip(_COUNTER_NAMES, (int(x) for x in out)))


# ---------------------------------------------------------------------------------------------
# Sharded simulator (C5): nodes partitioned over shards; a round = five stages + four message
# exchanges (include/ringpop_amd.h "Sharded simulator"). Bytes on the wire per message: a
# 40-byte header and 24-byte records.

MSG_BYTES = 40
REC_BYTES = 24
SIM_STAGES = 5


def shard_bounds(n, nshards):
    """Equal contiguous ranges (the C ABI's default partition)."""
    return np.array([n * g // nshards for g in range(nshards + 1)], dtype=np.uint32)


class SimShard:
    """One shard handle of the gossip simulator: nodes [v0, v0 + NL) with full views."""

    def __init__(self, names, inc0, dead, nshards, shard, seed=11, suspicion_rounds=25, now0=None, device=0,
                 bounds=None, events=()):
        self.N = len(names)
        self.G = nshards
        self.shard = shard
        self.dead = np.ascontiguousarray(dead, dtype=np.uint8)
        self.bounds = np.ascontiguousarray(bounds if bounds is not None else shard_bounds(self.N, nshards),
                                           dtype=np.uint32)
        self._h = _sim_create(names, inc0, self.dead, seed, suspicion_rounds, now0, device, self.bounds, nshards,
                              shard, events)
        self.v0 = int(self.bounds[shard])
        self.NL = int(self.bounds[shard + 1]) - self.v0

    def close(self):
        if getattr(self, "_h", None):
            lib().rp_sim_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stage(self, k):
        check(lib().rp_sim_stage(self._h, k))

    def join_export(self):
        """The round's events up to its next join (rp_sim_join_export): (has, device buffer,
        bytes) with this shard's responders' rows; the caller sums the shards' buffers."""
        has = ctypes.c_int()
        bp = ctypes.c_void_p()
        nb = ctypes.c_uint64()
        check(lib().rp_sim_join_export(self._h, ctypes.byref(has), ctypes.byref(bp), ctypes.byref(nb)))
        return bool(has.value), bp.value or 0, nb.value

    def join_import(self):
        check(lib().rp_sim_join_import(self._h))

    def outbox(self):
        """(nmsg[G], nrec[G], device buffer): per destination in shard order, a segment of
        nmsg[g] 40-byte headers then nrec[g] 24-byte records."""
        nm = np.zeros(self.G, dtype=np.uint64)
        nr = np.zeros(self.G, dtype=np.uint64)
        bp = ctypes.c_void_p()
        check(lib().rp_sim_outbox(self._h, nm.ctypes.data, nr.ctypes.data, ctypes.byref(bp)))
        return nm, nr, bp.value or 0

    def inbox(self, nmsg, nrec):
        """Size the inbox for per-source counts; returns its device buffer (to be filled with the
        sources' segments in source order)."""
        nm = np.ascontiguousarray(nmsg, dtype=np.uint64)
        nr = np.ascontiguousarray(nrec, dtype=np.uint64)
        bp = ctypes.c_void_p()
        check(lib().rp_sim_inbox(self._h, nm.ctypes.data, nr.ctypes.data, ctypes.byref(bp)))
        return bp.value or 0

    @property
    def round(self):
        v = ctypes.c_int64()
        check(lib().rp_sim_round(self._h, ctypes.byref(v)))
        return v.value

    def checksums(self):
        out = np.empty(self.NL, dtype=np.uint32)
        if self.NL:
            check(lib().rp_sim_checksums(self._h, out.ctypes.data))
        return out

    def view(self, v):
        st = np.empty(self.N, dtype=np.uint8)
        inc = np.empty(self.N, dtype=np.int64)
        check(lib().rp_sim_view(self._h, v, st.ctypes.data, inc.ctypes.data))
        return st, inc

    def conv_local(self):
        out = np.zeros(4, dtype=np.uint32)
        check(lib().rp_sim_converged_local(self._h, out.ctypes.data))
        return out

    def stats(self):
        out = np.zeros(4, dtype=np.uint64)
        check(lib().rp_sim_stats(self._h, out.ctypes.data))
        return out

    def piggyback(self):
        out = np.empty(self.NL, dtype=np.uint32)
        if self.NL:
            check(lib().rp_sim_piggyback(self._h, out.ctypes.data))
        return out

    def counters(self):
        out = np.zeros(8, dtype=np.uint64)
        check(lib().rp_sim_counters(self._h, out.ctypes.data))
        return out


def conv_reduce(parts):
    """Convergence (scenario-runner.js:152-170 + killed members faulty everywhere) from the
    shards' {live, min checksum, max checksum, killed-not-faulty} parts."""
    live = sum(int(p[0]) for p in parts)
    if live == 0:
        return True
    lo = min(int(p[1]) for p in parts if int(p[0]))
    hi = max(int(p[2]) for p in parts if int(p[0]))
    return lo == hi and not any(int(p[3]) for p in parts)


_STAT_NAMES = ["pings", "pingreqs", "fullsyncs", "applied"]
_COUNTER_NAMES = _STAT_NAMES + ["messages", "records", "views_hashed", "base_len"]


class ShardedGossipSim:
    """The simulator split into `nshards` shard handles inside this process (one device or
    several: `devices`), exchanging messages with device copies (rp_sim_exchange_local). Same
    results as GossipSim; used to test the sharded path on one GPU."""

    def __init__(self, names, inc0, dead, nshards, seed=11, suspicion_rounds=25, now0=None, devices=None,
                 bounds=None, events=()):
        self.N = len(names)
        self.G = nshards
        devices = devices or [0] * nshards
        self.shards = [SimShard(names, inc0, dead, nshards, g, seed, suspicion_rounds, now0, devices[g], bounds,
                                events) for g in range(nshards)]
        self._arr = (ctypes.c_void_p * nshards)(*[s._h.value for s in self.shards])

    def close(self):
        for s in self.shards:
            s.close()

    def _joins(self):
        """The round's join events (rp_sim_join_export / exchange / import, before stage 0)."""
        while True:
            has = [s.join_export()[0] for s in self.shards]
            if not any(has):
                return
            check(lib().rp_sim_join_exchange_local(self._arr, self.G))
            for s in self.shards:
                s.join_import()

    def step(self, rounds=1):
        for _ in range(rounds):
            self._joins()
            for k in range(SIM_STAGES):
                for s in self.shards:
                    s.stage(k)
                if k < SIM_STAGES - 1:
                    check(lib().rp_sim_exchange_local(self._arr, self.G))

    @property
    def round(self):
        return self.shards[0].round

    def checksums(self):
        return np.concatenate([s.checksums() for s in self.shards])

    def view(self, v):
        for s in self.shards:
            if s.v0 <= v < s.v0 + s.NL:
                return s.view(v)
        raise IndexError(v)

    def converged(self):
        return conv_reduce([s.conv_local() for s in self.shards])

    def stats(self):
        tot = sum(s.stats() for s in self.shards)
        return dict(zip(_STAT_NAMES, (int(x) for x in tot)))

    def counters(self):
        c = sum(s.counters() for s in self.shards)
        c[7] = self.shards[0].counters()[7]
        return dict(zip(_COUNTER_NAMES, (int(x) for x in c)))

    def piggyback(self):
        return np.concatenate([s.piggyback() for s in self.shards])


class _DeviceBytes:
    """A device byte range seen by torch without a copy (__cuda_array_interface__)."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": "|u1", "data": (int(ptr), False),
                                         "version": 2, "strides": None}


class MessageExchange:
    """All-to-all-v of the sharded simulator's messages over torch.distributed: one collective
    for the per-peer counts, one for the bytes. The simulator's outbox already holds one segment
    per destination ([40-byte headers | 24-byte records]) and its inbox takes one segment per
    source, so with the nccl backend (RCCL on ROCm) the collective reads the outbox and writes
    the inbox in HBM directly, over xGMI, with no staging copies. With gloo the bytes go through
    one host buffer each way (`copy(dst, src, nbytes)` moves them; tests)."""

    def __init__(self, group=None, device=None, copy=None, side_counts=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.G = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        backend = dist.get_backend(group)
        self.on_device = backend == "nccl"
        self.device = torch.device("cuda", device) if self.on_device and isinstance(device, int) else \
            (device if self.on_device else "cpu")
        self._copy = copy
        # the per-peer counts are host integers already (the outbox read), and all_to_all_single
        # takes its split sizes as host integers: with nccl they cross ranks over a gloo group of
        # the same ranks (no device collective, no device -> host read, round 5). side_counts
        # forces that side group on (gloo tests) or off. Every rank of `group` must construct the
        # exchange (the side group is built with local synchronization: ranks outside `group`
        # take no part).
        self._cgroup = None
        if self.on_device if side_counts is None else side_counts:
            self._cgroup = self._side_count_group()
        self._cdev = self.on_device and self._cgroup is None
        cdev = self.device if self._cdev else "cpu"
        if self._cgroup is None:
            self._cgroup = group
        self._cnt = torch.zeros(2 * self.G, dtype=torch.int64, device=cdev)
        self._rcnt = torch.zeros(2 * self.G, dtype=torch.int64, device=cdev)
        self._host = {}  # gloo staging buffers, kept across rounds
        self._events = []  # (start, end) of every byte collective queued on the device

    def _side_count_group(self):
        """A gloo group of this exchange's ranks for the per-peer counts, or None when any rank
        could not build one (every rank then counts over the main group: the choice is agreed
        by an all-reduce, so no two ranks ever use different count groups). Loopback is used
        only when every rank runs on this host (an all-gather of the host names' hashes), and
        only for the side group's creation: the process environment is restored."""
        import socket
        import zlib
        torch, dist, group = self.torch, self.dist, self.group
        ranks = list(range(self.G)) if group is None else dist.get_process_group_ranks(group)
        dev = self.device if self.on_device else "cpu"
        h = torch.tensor([zlib.crc32(socket.gethostname().encode())], dtype=torch.int64, device=dev)
        hs = [torch.empty_like(h) for _ in range(self.G)]
        dist.all_gather(hs, h, group=group)
        loopback = len({int(x.item()) for x in hs}) == 1 and "GLOO_SOCKET_IFNAME" not in os.environ
        cg = None
        try:
            if loopback:
                os.environ["GLOO_SOCKET_IFNAME"] = "lo"
            cg = dist.new_group(ranks=ranks, backend="gloo", use_local_synchronization=True)
        except Exception:  # no gloo here
            cg = None
        finally:
            if loopback:
                os.environ.pop("GLOO_SOCKET_IFNAME", None)
        ok = torch.tensor([0 if cg is None else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        return cg if int(ok.item()) == 1 else None

    def device_ms(self):
        """Device time of the byte collectives queued since the last call (nccl; 0 with gloo)."""
        if not self._events:
            return 0.0
        self._events[-1][1].synchronize()
        ms = sum(a.elapsed_time(b) for a, b in self._events)
        self._events = []
        return ms

    def copy(self, dst, src, nbytes):
        if nbytes:
            if self._copy is not None:
                self._copy(dst, src, nbytes)
            else:
                stream = self.torch.cuda.current_stream().cuda_stream if self.on_device else None
                check(lib().rp_copy(dst, src, nbytes, stream))

    def _staging(self, key, n):
        t = self._host.get(key)
        if t is None or t.numel() < n:
            t = self.torch.empty(max(n, 1) + max(n, 1) // 2, dtype=self.torch.uint8)
            self._host[key] = t
        return t

    def exchange(self, out_nmsg, out_nrec, out_buf, alloc_in, after=None, before=None):
        """out_*: this rank's outbox (counts per destination, its packed buffer's address).
        alloc_in(in_nmsg, in_nrec) -> the inbox's address, which receives every source's segment
        for this rank in source order. after(stream): with the nccl backend, called with torch's
        stream once the byte collective is queued on it, so the consumer orders its next work
        after it on the device (rp_sim_wait_stream); without it the host waits for the stream.
        before(stream): called once the inbox is sized, before the bytes move, with torch's stream
        (nccl) or None (gloo: the host is about to read the outbox), so that the reader waits for
        the producer's outbox fill and its last reads of the inbox (rp_sim_order_stream).
        The per-peer counts are host integers (torch's all_to_all_single takes its split sizes
        as host integers, and the inbox is sized from them); they cross ranks on the host (a gloo
        group beside the nccl one), so the exchange itself never waits for the device."""
        torch, dist, G = self.torch, self.dist, self.G
        self._cnt.copy_(torch.from_numpy(np.stack([out_nmsg, out_nrec], axis=1).astype(np.int64).reshape(-1)))
        dist.all_to_all_single(self._rcnt, self._cnt, group=self._cgroup)
        rc = (self._rcnt.cpu() if self._cdev else self._rcnt).numpy().reshape(G, 2)
        in_nmsg, in_nrec = rc[:, 0].astype(np.uint64), rc[:, 1].astype(np.uint64)
        seg_out = [int(out_nmsg[g]) * MSG_BYTES + int(out_nrec[g]) * REC_BYTES for g in range(G)]
        seg_in = [int(in_nmsg[g]) * MSG_BYTES + int(in_nrec[g]) * REC_BYTES for g in range(G)]
        tot_out, tot_in = sum(seg_out), sum(seg_in)
        in_buf = alloc_in(in_nmsg, in_nrec)
        if before is not None:
            before(torch.cuda.current_stream().cuda_stream if self.on_device else None)
        if self.on_device:
            send = torch.as_tensor(_DeviceBytes(out_buf, tot_out), device=self.device) if tot_out else \
                torch.empty(0, dtype=torch.uint8, device=self.device)
            recv = torch.as_tensor(_DeviceBytes(in_buf, tot_in), device=self.device) if tot_in else \
                torch.empty(0, dtype=torch.uint8, device=self.device)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dist.all_to_all_single(recv, send, output_split_sizes=seg_in, input_split_sizes=seg_out,
                                   group=self.group)
            e1.record()
            self._events.append((e0, e1))
            if after is not None:
                after(torch.cuda.current_stream().cuda_stream)
            else:
                torch.cuda.current_stream().synchronize()
        else:
            send = self._staging("send", tot_out)
            recv = self._staging("recv", tot_in)
            self.copy(send.data_ptr(), out_buf, tot_out)
            dist.all_to_all_single(recv[:tot_in], send[:tot_out], output_split_sizes=seg_in,
                                   input_split_sizes=seg_out, group=self.group)
            self.copy(in_buf, recv.data_ptr(), tot_in)
        return in_nmsg, in_nrec

    def sum_bytes(self, buf, nbytes, after=None):
        """Byte-wise sum of every rank's device buffer into each rank's (the join exchange).
        after(stream): as in exchange (nccl: the consumer waits on the device, not the host)."""
        torch, dist = self.torch, self.dist
        if self.on_device:
            t = torch.as_tensor(_DeviceBytes(buf, nbytes), device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            if after is not None:
                after(torch.cuda.current_stream().cuda_stream)
            else:
                torch.cuda.current_stream().synchronize()
        else:
            h = self._staging("join", nbytes)
            self.copy(h.data_ptr(), buf, nbytes)
            v = h[:nbytes]
            dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.group)
            self.copy(buf, h.data_ptr(), nbytes)


class DistGossipSim:
    """One shard of the simulator per torch.distributed rank (C5 over 1/2/4/8 GPUs: views
    sharded by node id range, the four per-round message exchanges as RCCL all-to-all-v).
    Results equal GossipSim's on the same inputs."""

    def __init__(self, names, inc0, dead, seed=11, suspicion_rounds=25, now0=None, device=0, group=None, events=()):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.xchg = MessageExchange(group, device=device)
        self.G, self.rank = self.xchg.G, self.xchg.rank
        self.N = len(names)
        self.shard = SimShard(names, inc0, dead, self.G, self.rank, seed, suspicion_rounds, now0, device,
                              events=events)
        self.exchange_bytes = 0
        # host wall time inside the exchanges (count all-to-all + its host read, inbox sizing, the
        # byte all-to-all-v queued, and the join sums): what the message transport adds to a round
        self.exchange_s = 0.0

    def close(self):
        self.shard.close()

    def step(self, rounds=1):
        import time
        sh = self.shard
        wait = lambda stream: check(lib().rp_sim_wait_stream(sh._h, stream))  # noqa: E731
        order = lambda stream: check(lib().rp_sim_order_stream(sh._h, stream))  # noqa: E731
        for _ in range(rounds):
            while True:  # the round's joins: every rank exports, the buffers are summed, then import
                has, buf, nb = sh.join_export()
                if not has:
                    break
                t = time.perf_counter()
                self.xchg.sum_bytes(buf, nb, after=wait)
                self.exchange_s += time.perf_counter() - t
                sh.join_import()
            for k in range(SIM_STAGES):
                sh.stage(k)
                if k < SIM_STAGES - 1:
                    nm, nr, buf = sh.outbox()
                    self.exchange_bytes += int(nm.sum()) * MSG_BYTES + int(nr.sum()) * REC_BYTES
                    t = time.perf_counter()
                    self.xchg.exchange(nm, nr, buf, sh.inbox, after=wait, before=order)
                    self.exchange_s += time.perf_counter() - t

    @property
    def round(self):
        return self.shard.round

    def _allgather(self, arr):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr))
        if self.xchg.on_device:
            t = t.to(self.xchg.device)
        outs = [torch.empty_like(t) for _ in range(self.G)]
        self.dist.all_gather(outs, t, group=self.group)
        return [o.cpu().numpy() for o in outs]

    def converged(self):
        return conv_reduce(self._allgather(self.shard.conv_local().astype(np.int64)))

    def checksums(self):
        """All N checksums (gathered; shards may differ in size)."""
        sizes = np.diff(self.shard.bounds.astype(np.int64))
        mx = int(sizes.max())
        mine = np.zeros(mx, dtype=np.int64)
        mine[:self.shard.NL] = self.shard.checksums()
        parts = self._allgather(mine)
        return np.concatenate([p[:int(n)] for p, n in zip(parts, sizes)]).astype(np.uint32)

    def stats(self):
        tot = sum(self._allgather(self.shard.stats().astype(np.int64)))
        return dict(zip(_STAT_NAMES, (int(x) for x in tot)))

    def counters(self):
        c = sum(self._allgather(self.shard.counters().astype(np.int64)))
        c[7] = self.shard.counters()[7]
        return dict(zip(_COUNTER_NAMES, (int(x) for x in c)))


# ------------------------------------------------------------------ gossip wire bodies
# Device JSON codec of change records (rp_wire_*_dev): dissemination.js:163-170 / 64-73 records,
# ping bodies ping-sender.js:71-76 and server/protocol/ping.js:45-48. torch is only the device
# buffer plumbing here.
WIRE_FORM = {"issueAs": 0, "fullSync": 1}
WIRE_BODY = {"array": 0, "ping": 1, "pingResponse": 2, "pingReq": 3, "pingReqResponse": 4, "joinResponse": 5}
INT64_MIN = -(1 << 63)


class WireRecords(ctypes.Structure):
    """rp_wire_records (include/ringpop_amd.h)."""
    _fields_ = [("addr", _P), ("src", _P), ("status", _P), ("inc", _P), ("src_inc", _P), ("ids", _P)]


class WireHeaders(ctypes.Structure):
    """rp_wire_headers."""
    _fields_ = [("checksum", _P), ("source", _P), ("source_inc", _P), ("target", _P), ("ping_status", _P),
                ("app", ctypes.c_char_p), ("app_len", _U32)]


class WireRecordsOut(ctypes.Structure):
    """rp_wire_records_out."""
    _fields_ = [("addr", _P), ("src", _P), ("status", _P), ("inc", _P), ("src_inc", _P), ("id_off", _P),
                ("addr_off", _P), ("addr_len", _P)]


class WireHeadersOut(ctypes.Structure):
    """rp_wire_headers_out."""
    _fields_ = [("checksum", _P), ("source", _P), ("source_inc", _P), ("target", _P), ("ping_status", _P)]


def _dev(a, dtype):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=dtype).copy()).cuda()


def wire_encode(members, msg_rec_off, addr, src, status, inc, src_inc=None, ids=None, form="issueAs",
                body="array", msg_checksum=None, msg_source=None, msg_source_inc=None, msg_target=None,
                msg_ping_status=None, app=None):
    """Encode message j = records [msg_rec_off[j], msg_rec_off[j+1]) on the device; returns
    (bytes, out_off) on the host. addr/src/msg_source/msg_target are ids interned in `members`
    (src NULL_ID = no source member); src_inc None or INT64_MIN entries = absent; ids is an
    (n_rec, 36) uint8 array of uuid strings (a row starting with 0 = absent) or None."""
    import torch
    n_msgs = len(msg_rec_off) - 1
    n_rec = len(addr)
    d = dict(off=_dev(msg_rec_off, np.uint32), addr=_dev(addr if n_rec else [0], np.uint32),
             src=_dev(src if n_rec else [0], np.uint32), st=_dev(status if n_rec else [0], np.uint8),
             inc=_dev(inc if n_rec else [0], np.int64))
    d["sinc"] = _dev(src_inc, np.int64) if src_inc is not None and n_rec else None
    d["ids"] = _dev(np.asarray(ids, dtype=np.uint8).reshape(-1), np.uint8) if ids is not None and n_rec else None
    col = lambda x, dt: None if x is None or n_msgs == 0 else _dev(x, dt)  # noqa: E731
    h = dict(ck=col(msg_checksum, np.uint32), ms=col(msg_source, np.uint32), msi=col(msg_source_inc, np.int64),
             tg=col(msg_target, np.uint32), ps=col(msg_ping_status, np.uint8))
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    recs = WireRecords(p(d["addr"]), p(d["src"]), p(d["st"]), p(d["inc"]), p(d["sinc"]), p(d["ids"]))
    appb = (app.encode() if isinstance(app, str) else app) if app is not None else None
    hdr = WireHeaders(p(h["ck"]), p(h["ms"]), p(h["msi"]), p(h["tg"]), p(h["ps"]), appb, len(appb or b""))
    stream = torch.cuda.current_stream().cuda_stream
    out_off = torch.empty(n_msgs + 1, dtype=torch.int64, device="cuda")
    args = [members._h, n_msgs, p(d["off"]), n_rec, ctypes.byref(recs), WIRE_FORM[form], WIRE_BODY[body],
            ctypes.byref(hdr)]
    check(lib().rp_wire_encode_dev(*args, None, out_off.data_ptr(), stream))
    total = int(out_off[-1].item())
    out = torch.empty(max(total, 1), dtype=torch.uint8, device="cuda")
    check(lib().rp_wire_encode_dev(*args, out.data_ptr(), out_off.data_ptr(), stream))
    return out[:total].cpu().numpy().tobytes(), out_off.cpu().numpy().astype(np.uint64)


def wire_decode(members, texts):
    """Decode JSON texts (changes arrays or any of the bodies) on the device. Returns a dict of
    numpy columns: rec_off, addr, src, status, inc, src_inc, id_off, addr_off, addr_len, err and
    the per-message checksum / source / source_inc / target / ping_status."""
    import torch
    texts = [t.encode() if isinstance(t, str) else bytes(t) for t in texts]
    n = len(texts)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(t) for t in texts])
    buf = _dev(np.frombuffer(b"".join(texts) or b"\0", dtype=np.uint8).copy(), np.uint8)
    d_off = _dev(off, np.uint64)
    cap = max(sum(t.count(b"{") for t in texts), 1)
    e = lambda dt, k=cap: torch.empty(k, dtype=dt, device="cuda")  # noqa: E731
    m1 = max(n, 1)
    c = dict(rec_off=e(torch.int32, n + 1), addr=e(torch.int32), src=e(torch.int32), status=e(torch.uint8),
             inc=e(torch.int64), src_inc=e(torch.int64), id_off=e(torch.int64), addr_off=e(torch.int64),
             addr_len=e(torch.int32), err=e(torch.int64, m1), checksum=e(torch.int32, m1),
             source=e(torch.int32, m1), source_inc=e(torch.int64, m1), target=e(torch.int32, m1),
             ping_status=e(torch.uint8, m1))
    p = {k: v.data_ptr() for k, v in c.items()}
    recs = WireRecordsOut(p["addr"], p["src"], p["status"], p["inc"], p["src_inc"], p["id_off"], p["addr_off"],
                          p["addr_len"])
    hdr = WireHeadersOut(p["checksum"], p["source"], p["source_inc"], p["target"], p["ping_status"])
    check(lib().rp_wire_decode_dev(members._h, buf.data_ptr(), d_off.data_ptr(), n, p["rec_off"], cap,
                                   ctypes.byref(recs), ctypes.byref(hdr), p["err"],
                                   torch.cuda.current_stream().cuda_stream))
    h = {k: v.cpu().numpy() for k, v in c.items()}
    k = int(h["rec_off"][n])
    u32 = lambda a: a.view(np.uint32)  # noqa: E731
    return dict(rec_off=u32(h["rec_off"]), addr=u32(h["addr"])[:k], src=u32(h["src"])[:k], status=h["status"][:k],
                inc=h["inc"][:k], src_inc=h["src_inc"][:k], id_off=h["id_off"][:k].view(np.uint64),
                addr_off=h["addr_off"][:k], addr_len=h["addr_len"][:k], err=h["err"][:n],
                checksum=u32(h["checksum"])[:n], source=u32(h["source"])[:n], source_inc=h["source_inc"][:n],
                target=u32(h["target"])[:n], ping_status=h["ping_status"][:n])
