"""CPU tests of the Node N-API addon (ringpop-node_amd/js): it builds, loads in node, exports
every entry point index.js uses, its hash32 is the engine's farmhash32 (checked against the
oracle), and without a device the reference-API classes refuse to construct (no fallback)."""
import json
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(REPO, "ringpop-node_amd", "js")
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None or not os.path.isdir("/usr/include/node"),
                                reason="node / N-API headers not in this image")

EXPORTS = ["version", "deviceCount", "hash32", "destroy", "ringCreate", "ringAddRemove", "ringChecksum",
           "ringChecksumString", "ringServerCount", "ringService", "ringLookup1", "ringLookupN1", "ringTokenCount", "ringHasServer", "ringServers",
           "ringOwnerName", "ringLookup", "ringLookupN", "ringLookupNHashes", "ringGroupKeys", "membersCreate", "membersIntern",
           "membersSetLocal", "membersUpdate", "membersSet", "membersChecksum", "membersComputeChecksum",
           "membersChecksumString", "membersDump", "membersDampConfigure", "membersDampLast", "membersDampDecay",
           "membersDampDump", "simCreate", "simStep", "simRound", "simChecksums",
           "simView", "simConverged", "simStats", "wireEncode", "wireDecode"]


@pytest.fixture(scope="module")
def addon(rpa):
    subprocess.check_call(["make", "-s", "-C", JS])
    return os.path.join(JS, "rpamd.node")


def node(script, *args):
    out = subprocess.run([NODE, "-e", script, *args], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return out.stdout


def test_addon_exports(addon):
    got = json.loads(node("console.log(JSON.stringify(Object.keys(require(process.argv[1]))))", addon))
    assert sorted(got) == sorted(EXPORTS)


def test_addon_hash32_matches_oracle(addon, orc):
    keys = ["", "a", "ab", "abc", "abcd", "10.0.0.1:20800", "127.0.0.1:3000" + "0", "x" * 100,
            "héllo wörld", "ÿ" * 33] + ["k%d" % i for i in range(200)]
    got = json.loads(node("var a=require(process.argv[1]);var k=JSON.parse(process.argv[2]);"
                          "console.log(JSON.stringify(k.map(a.hash32)))", addon, json.dumps(keys)))
    assert got == [orc.hash32(k.encode()) for k in keys]


def test_no_device_refuses(addon, rpa):
    if rpa.device_count() > 0:
        pytest.skip("a device is visible")
    out = node("var amd=require(process.argv[1]);"
               "try{new amd.HashRing();console.log('constructed')}catch(e){console.log('refused: '+e.message)}",
               os.path.join(JS, "index.js"))
    assert out.startswith("refused: ringpop_amd: no HIP device"), out
