// svc_latency.js — the resident lookup service's per-call latency alone (round 5 A/B):
// HashRing.lookup / lookupN(3) one key at a time on the C2 ring through rp_ring_service, under
// whatever RP_RING_SVC / RP_SVC_POLLS / RP_SVC_WARM / RP_SVC_PROF the caller set; the
// service's own phase breakdown (RP_SVC_PROF) goes to stderr when the service stops.
//   node tools/svc_latency.js [servers=10000] [calls=3000] [distinct keys=8192]
'use strict';
var path = require('path');
var crypto = require('crypto');
var amd = require(path.join(__dirname, '..', 'ringpop-node_amd', 'js'));
var nServers = parseInt(process.argv[2] || '10000', 10);
var calls = parseInt(process.argv[3] || '3000', 10);
var nKeys = parseInt(process.argv[4] || '8192', 10);
function addr(i) { return '10.' + ((i >> 16) & 255) + '.' + ((i >> 8) & 255) + '.' + (i & 255) + ':' + (20800 + i % 36); }
function uuid() {
    var h = crypto.randomBytes(16).toString('hex');
    return h.slice(0, 8) + '-' + h.slice(8, 12) + '-' + h.slice(12, 16) + '-' + h.slice(16, 20) + '-' + h.slice(20);
}
function now() { return Number(process.hrtime.bigint()) / 1e3; }
function timeit(fn, n, w) {
    for (var i = 0; i < w; i++) { fn(i); }
    var t = [];
    for (var j = 0; j < n; j++) { var a = now(); fn(j); t.push(now() - a); }
    t.sort(function (x, y) { return x - y; });
    return {median_us: t[t.length >> 1], p10_us: t[Math.floor(t.length * 0.1)], p90_us: t[Math.floor(t.length * 0.9)], calls: n};
}
var ring = new amd.HashRing();
var servers = [];
for (var s = 0; s < nServers; s++) { servers.push(addr(s)); }
ring.addRemoveServers(servers);
var keys = [];
for (var k = 0; k < nKeys; k++) { keys.push(uuid()); }
var out = {env: {RP_RING_SVC: process.env.RP_RING_SVC || '2', RP_SVC_WAVES: process.env.RP_SVC_WAVES || '8',
                 RP_SVC_PERIOD: process.env.RP_SVC_PERIOD || '120', RP_SVC_WARM: process.env.RP_SVC_WARM || '0'},
           keys: nKeys};
amd.native.ringService(ring._h, 2000);
out.lookup_service = timeit(function (i) { ring.lookup(keys[i % keys.length]); }, calls, 300);
amd.native.ringService(ring._h, 0);
amd.native.ringService(ring._h, 2000);
out.lookupN3_service = timeit(function (i) { ring.lookupN(keys[i % keys.length], 3); }, calls, 300);
amd.native.ringService(ring._h, 0);
console.log(JSON.stringify(out));
