// ref_ring_ops.js — runs the REFERENCE HashRing (lib/ring/index.js, read from the reference
// checkout given on the command line) over sequences of single calls (addServer, removeServer,
// addRemoveServers, hasServer) and records each call's return value, the events it emitted,
// and the ring's checksum, server count, Object.keys(servers) and tree size after it.
// Golden-vector generator only (tests/golden/make_ring_ops.py); never shipped, never run on the
// GPU box.
//
//   NODE_PATH=oracle/_ref/node_modules node tests/golden/ref_ring_ops.js <ref_root> <in.json> <out.json>
'use strict';
var fs = require('fs');
var path = require('path');

var refRoot = process.argv[2];
var input = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
var HashRing = require(path.join(refRoot, 'lib/ring'));

var out = {cases: []};
input.cases.forEach(function (c) {
    var ring = new HashRing(c.replicaPoints ? {replicaPoints: c.replicaPoints} : {});
    var events = [];
    ['added', 'removed', 'checksumComputed'].forEach(function (e) {
        ring.on(e, function (name) { events.push(name === undefined ? e : e + ':' + name); });
    });
    var co = {name: c.name, ops: []};
    c.ops.forEach(function (op) {
        events.length = 0;
        var ret = ring[op[0]].apply(ring, op.slice(1));
        co.ops.push({ret: ret === undefined ? null : ret, events: events.slice(), checksum: ring.checksum,
                     serverCount: ring.getServerCount(), servers: Object.keys(ring.servers),
                     size: ring.rbtree.size});
    });
    out.cases.push(co);
});
fs.writeFileSync(process.argv[4], JSON.stringify(out));
