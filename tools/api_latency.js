// api_latency.js — per-call latency of the drop-in JS API on the device (bench.py's api_latency
// leg; node on the GPU box). The reference's own API is called one key / one ping's changes at
// a time: RingPop.lookup / lookupN (index.js:434-471 -> lib/ring/index.js:145-189) and the
// per-ping Membership.update (server/protocol/ping.js:44 -> lib/membership/index.js:249-324).
// Through rpamd.node each such call is a launch plus a host round trip; this times those forms
// and the batched ones, so the batch size where the device wins can be read off.
//
//   node tools/api_latency.js [servers=10000] [members=100000,10000,1332]
// Prints one JSON line.
'use strict';
var path = require('path');
var crypto = require('crypto');
var EventEmitter = require('events').EventEmitter;
var util = require('util');
var amd = require(path.join(__dirname, '..', 'ringpop-node_amd', 'js'));
var drop = require(path.join(__dirname, '..', 'ringpop-node_amd', 'js', 'membership.js'));

var nServers = parseInt(process.argv[2] || '10000', 10);
var memberSizes = (process.argv[3] || '100000,10000,1332').split(',').map(function (x) { return parseInt(x, 10); });

function addr(i) {  // SURVEY §8d C2 address
    return '10.' + ((i >> 16) & 255) + '.' + ((i >> 8) & 255) + '.' + (i & 255) + ':' + (20800 + i % 36);
}
function uuid() {
    var h = crypto.randomBytes(16).toString('hex');
    return h.slice(0, 8) + '-' + h.slice(8, 12) + '-' + h.slice(12, 16) + '-' + h.slice(16, 20) + '-' + h.slice(20);
}
function now() { return Number(process.hrtime.bigint()) / 1e3; }  // µs

// median µs per call of fn(i) over n calls after w warm-up calls
function timeit(fn, n, w) {
    for (var i = 0; i < w; i++) { fn(i); }
    var t = [];
    for (var j = 0; j < n; j++) {
        var a = now();
        fn(j);
        t.push(now() - a);
    }
    t.sort(function (x, y) { return x - y; });
    return {median_us: t[t.length >> 1], p90_us: t[Math.floor(t.length * 0.9)], calls: n};
}

var out = {servers: nServers};
var ring = new amd.HashRing({serviceIdleMs: 0});  // the launch-per-call legs first; the service below
var servers = [];
for (var s = 0; s < nServers; s++) { servers.push(addr(s)); }
ring.addRemoveServers(servers);
var keys = [];
for (var k = 0; k < 8192; k++) { keys.push(uuid()); }
out.lookup = timeit(function (i) { ring.lookup(keys[i % keys.length]); }, 2000, 200);
out.lookupN3 = timeit(function (i) { ring.lookupN(keys[i % keys.length], 3); }, 2000, 200);
// the same single calls through the resident lookup service (rp_ring_service)
native_service: {
    amd.native.ringService(ring._h, 2000);
    out.lookup_service = timeit(function (i) { ring.lookup(keys[i % keys.length]); }, 2000, 200);
    out.lookupN3_service = timeit(function (i) { ring.lookupN(keys[i % keys.length], 3); }, 2000, 200);
    amd.native.ringService(ring._h, 0);
}
out.lookupNBatch3 = {};
[1, 64, 4096].forEach(function (b) {
    var r = timeit(function (i) { ring.lookupNBatch(keys.slice((i * b) % 4096, (i * b) % 4096 + b), 3); }, b > 64 ? 200 : 1000, 50);
    r.us_per_key = r.median_us / b;
    out.lookupNBatch3[b] = r;
});
// per-call ring mutation on the C2 ring, the call pattern of lib/on_membership_event.js:106-134
// (one applied alive / faulty / leave update -> ring.addRemoveServers with a handful of names):
// addServer of a new name, removeServer of it again, and addRemoveServers([new], [old]) that
// swaps one server (then swaps it back), each a device sort + merge + checksum
var extra = [];
for (var x = 0; x < 64; x++) { extra.push(addr(nServers + 1000 + x)); }
out.addServer = timeit(function (i) { ring.addServer(extra[i % 64]); ring.removeServer(extra[i % 64]); }, 100, 5);
out.addServer.note = 'one addServer + one removeServer per call';
out.addServer.median_us_per_mutation = out.addServer.median_us / 2;
out.addRemoveServers = timeit(function (i) {
    var a = extra[i % 64], b = servers[(i * 7919) % nServers];
    ring.addRemoveServers([a], [b]);
    ring.addRemoveServers([b], [a]);
}, 100, 5);
out.addRemoveServers.note = 'two addRemoveServers([a], [b]) calls per timed call';
out.addRemoveServers.median_us_per_mutation = out.addRemoveServers.median_us / 2;
ring.destroy();

// the drop-in Membership (js/membership.js) with a stand-in ringpop, n members, then ping-sized
// update batches of fresh incarnations (every change applies; each applied batch computes the
// checksum, as the reference's does)
function FakeRingpop(whoami) {
    EventEmitter.call(this);
    this.hostPort = whoami;
    this.isReady = true;
    this.logger = {debug: function () {}, info: function () {}, warn: function () {}, error: function () {}};
    this.config = {get: function (key) { return {dampScoringEnabled: false, dampScoringDecayEnabled: false}[key]; }};
}
util.inherits(FakeRingpop, EventEmitter);
FakeRingpop.prototype.whoami = function () { return this.hostPort; };
FakeRingpop.prototype.stat = function () {};

out.membershipUpdate = {};
memberSizes.forEach(function (n) {
    var rp = new FakeRingpop(addr(0));
    var m = drop.initMembership(rp, {capacity: n});
    rp.membership = m;
    // join positions: appended (the reference draws Math.random, index.js:129-131; a random
    // splice per new member is O(N^2) in JS and is not what is timed here)
    m.getJoinPosition = function () { return this.members.length; };
    var base = 1434401518824;
    var all = [];
    for (var i = 0; i < n; i++) { all.push({address: addr(i), status: 'alive', incarnationNumber: base}); }
    var t0 = now();
    m.update(all);
    var create = now() - t0;
    var inc = base;
    var res = {members: n, create_ms: create / 1e3};
    [1, 10, 100].forEach(function (c) {
        var r = timeit(function (j) {
            inc++;
            var ch = [];
            for (var q = 0; q < c; q++) {
                ch.push({address: addr((j * 7919 + q * 104729 + 1) % n), status: 'alive', incarnationNumber: inc});
            }
            m.update(ch);
        }, c === 100 ? 100 : 200, 10);
        res[c] = r;
    });
    m.destroy();
    out.membershipUpdate[n] = res;
});
process.stdout.write(JSON.stringify(out) + '\n');
