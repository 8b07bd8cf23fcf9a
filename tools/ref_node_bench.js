// ref_node_bench.js — times the REFERENCE JavaScript (lib/ring/index.js HashRing with its
// RBTree; lib/membership/index.js Membership.update + computeChecksum) on this host, single
// threaded (Node's event loop), for BASELINE.md: the reference's own CPU path at C1, C2 and C3.
// `farmhash` is the oracle's N-API restatement (oracle/_ref), underscore / node-uuid the minimal
// shims of oracle/gen/shims. Measurement tool only: it needs /root/reference, never runs on the
// GPU box.
//
//   NODE_PATH=oracle/_ref/node_modules node tools/ref_node_bench.js <ref_root> <in.json> <out.json>
'use strict';
var fs = require('fs');
var path = require('path');
var EventEmitter = require('events').EventEmitter;
var util = require('util');

var refRoot = process.argv[2];
var input = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
var HashRing = require(path.join(refRoot, 'lib/ring/index.js'));
var initMembership = require(path.join(refRoot, 'lib/membership/index.js'));

function now() { var t = process.hrtime(); return t[0] + t[1] * 1e-9; }

function FakeRingpop(whoami) {
    EventEmitter.call(this);
    this.hostPort = whoami;
    this.isReady = true;
    this.logger = {debug: function () {}, info: function () {}, warn: function () {}, error: function () {}};
    this.config = {get: function (k) {
        return {dampScoringEnabled: false, dampScoringDecayEnabled: false, dampScoringInitial: 0}[k];
    }};
}
util.inherits(FakeRingpop, EventEmitter);
FakeRingpop.prototype.whoami = function () { return this.hostPort; };
FakeRingpop.prototype.stat = function () {};

var out = {node: process.version, results: {}};

function ringCase(name, c) {
    var r = {};
    var ring = new HashRing();
    var t0 = now();
    ring.addRemoveServers(c.servers, []);
    r.build_ms = (now() - t0) * 1e3;
    var keys = c.keys;
    t0 = now();
    var sink = 0;
    for (var i = 0; i < keys.length; i++) { if (ring.lookup(keys[i]) !== null) { sink++; } }
    var dt = now() - t0;
    r.lookup = {keys: keys.length, per_s: keys.length / dt, seconds: dt};
    var nn = Math.min(keys.length, c.lookupNKeys);
    t0 = now();
    for (i = 0; i < nn; i++) { sink += ring.lookupN(keys[i], 3).length; }
    dt = now() - t0;
    r.lookupN3 = {keys: nn, per_s: nn / dt, seconds: dt};
    // per-call mutation (the call pattern of lib/on_membership_event.js:106-134): addServer +
    // removeServer of a new name, and addRemoveServers([new], [old]) swapping one server and back
    var extra = c.extra || [];
    if (extra.length) {
        var reps = extra.length;
        t0 = now();
        for (i = 0; i < reps; i++) { ring.addServer(extra[i]); ring.removeServer(extra[i]); }
        r.add_remove_server_ms_per_mutation = (now() - t0) * 1e3 / (2 * reps);
        t0 = now();
        for (i = 0; i < reps; i++) {
            var b = c.servers[(i * 7919) % c.servers.length];
            ring.addRemoveServers([extra[i]], [b]);
            ring.addRemoveServers([b], [extra[i]]);
        }
        r.addRemoveServers_swap_ms_per_call = (now() - t0) * 1e3 / (2 * reps);
        r.mutation_calls = 2 * reps;
    }
    r.sink = sink;
    out.results[name] = r;
}

function membershipCase(name, c) {
    var r = {};
    var rp = new FakeRingpop(c.names[0]);
    var m = initMembership(rp);
    rp.membership = m;
    var t0 = now();
    m.makeAlive(c.names[0], c.inc0[0]);
    m.update(c.names.slice(1).map(function (a, i) {
        return {address: a, status: 'alive', incarnationNumber: c.inc0[i + 1]};
    }));
    r.create_ms = (now() - t0) * 1e3;
    var ST = ['alive', 'suspect', 'faulty', 'leave'];
    var done = 0, applied = 0;
    t0 = now();
    c.batches.forEach(function (b, j) {
        var changes = b.ids.map(function (id, i) {
            return {address: c.names[id], status: ST[b.st[i]], incarnationNumber: b.inc[i]};
        });
        applied += m.update(changes).length;
        done += changes.length;
    });
    var dt = now() - t0;
    r.update = {batches: c.batches.length, updates: done, applied: applied, per_s: done / dt, seconds: dt,
                ms_per_batch: dt * 1e3 / c.batches.length};
    t0 = now();
    for (var k = 0; k < 5; k++) { m.computeChecksum(); }
    r.checksum_ms = (now() - t0) * 1e3 / 5;
    r.checksum = m.checksum;
    out.results[name] = r;
}

input.rings.forEach(function (c) { ringCase(c.name, c); });
input.memberships.forEach(function (c) { membershipCase(c.name, c); });
fs.writeFileSync(process.argv[4], JSON.stringify(out));
