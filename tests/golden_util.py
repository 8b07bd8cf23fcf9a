"""Helpers to replay tests/golden/*.json fixtures (data produced by the reference JS)."""
import json
import os

import pyoracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def hash_func(case):
    """The hashFunc the generator injected (tests/golden/ref_ring.js makeHash)."""
    kind = case["hashKind"]
    if kind == "farmhash":
        return None
    if kind == "port":
        return lambda s: int(s[s.rfind(":") + 1:])
    mod = case["hashMod"]
    return lambda s: int(s[1:]) if s.startswith("#") else pyoracle.hash32(s) % mod


def keys_of(batch):
    keys = batch["keys"]
    if isinstance(keys, dict):
        seed, k0, n = keys["uuid"]
        return [k.tobytes().decode() for k in pyoracle.uuid_keys(seed, k0, n)]
    return keys
