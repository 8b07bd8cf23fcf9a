// ref_ring.js — runs the REFERENCE HashRing (lib/ring/index.js + lib/ring/rbtree.js, read
// from the reference checkout given on the command line) over the cases in <in.json> and
// writes what it observed to <out.json>. Golden-vector generator only (tests/golden/make_golden.py);
// never shipped, never run on the GPU box.
//
//   NODE_PATH=oracle/_ref/node_modules node tests/golden/ref_ring.js <ref_root> <in.json> <out.json>
//
// `farmhash` resolves to the oracle's N-API restatement (oracle/gen/farmhash_napi.c).
// Custom hash functions go through the reference's own injection point
// `new HashRing({hashFunc})` (lib/ring/index.js:29).
'use strict';
var fs = require('fs');
var path = require('path');
var farmhash = require('farmhash');

var refRoot = process.argv[2];
var input = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
var HashRing = require(path.join(refRoot, 'lib/ring'));

function makeHash(kind, mod) {
    if (kind === 'farmhash') {
        return farmhash.hash32;
    }
    if (kind === 'port') {
        // test/unit/ring-test.js:32-34 extractPort
        return function extractPort(s) { return parseInt(s.substr(s.lastIndexOf(':') + 1)); };
    }
    // 'mod': '#<n>' probes hash to n; anything else to farmhash % mod (forces collisions)
    return function modHash(s) {
        if (s.charAt(0) === '#') { return parseInt(s.slice(1), 10); }
        return farmhash.hash32(s) % mod;
    };
}

function dumpTree(ring) {
    var toks = [], owners = [];
    var it = ring.rbtree.iterator();
    while (it.next() !== null) { toks.push(it.val()); owners.push(it.str()); }
    return {tokens: toks, owners: owners};
}

var out = {cases: []};
input.cases.forEach(function (c) {
    var opts = {};
    if (c.replicaPoints) { opts.replicaPoints = c.replicaPoints; }
    if (c.hashKind !== 'farmhash') { opts.hashFunc = makeHash(c.hashKind, c.hashMod); }
    var ring = new HashRing(opts);
    var co = {name: c.name, batches: []};
    c.batches.forEach(function (b) {
        var changed = ring.addRemoveServers(b.add, b.remove);
        var bo = {
            changed: changed,
            checksum: ring.checksum,
            serverCount: ring.getServerCount(),
            servers: Object.keys(ring.servers),
            size: ring.rbtree.size,
        };
        if (c.dump) { bo.tree = dumpTree(ring); }
        if (b.keys) {
            bo.lookup = b.keys.map(function (k) { return ring.lookup(k); });
            bo.lookupN = {};
            (b.ns || []).forEach(function (n) {
                bo.lookupN[String(n)] = b.keys.map(function (k) { return ring.lookupN(k, n); });
            });
        }
        co.batches.push(bo);
    });
    out.cases.push(co);
});
fs.writeFileSync(process.argv[4], JSON.stringify(out));
