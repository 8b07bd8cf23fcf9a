// ring_ops_parity.js — replays tests/golden/ring_ops_golden.json (single HashRing calls on the
// reference's lib/ring/index.js, inherited names such as 'constructor' included) through the
// N-API HashRing of ringpop-node_amd/js: each call's return value, events, checksum, server
// count (host map and device), Object.keys(servers). Prints one JSON line.
'use strict';
var fs = require('fs');
var path = require('path');
var amd = require(path.join(__dirname, '..', '..', 'ringpop-node_amd', 'js'));

var input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
var fails = [];
var checks = 0;

function eq(what, got, want) {
    checks++;
    if (JSON.stringify(got) !== JSON.stringify(want)) {
        fails.push({what: what, got: String(JSON.stringify(got)).slice(0, 200), want: String(JSON.stringify(want)).slice(0, 200)});
    }
}

input.cases.forEach(function (c) {
    var ring = new amd.HashRing(c.replicaPoints ? {replicaPoints: c.replicaPoints} : {});
    var events = [];
    ['added', 'removed', 'checksumComputed'].forEach(function (e) {
        ring.on(e, function (name) { events.push(name === undefined ? e : e + ':' + name); });
    });
    c.ops.forEach(function (op, i) {
        var tag = c.name + '#' + i + ' ' + JSON.stringify(op);
        var want = c.results[i];
        events.length = 0;
        var ret;
        try {
            ret = ring[op[0]].apply(ring, op.slice(1));
        } catch (e) {
            fails.push({what: tag + ' threw', got: String(e.message).slice(0, 200), want: JSON.stringify(want.ret)});
            return;
        }
        eq(tag + ' ret', ret === undefined ? null : ret, want.ret);
        eq(tag + ' events', events, want.events);
        eq(tag + ' checksum', ring.checksum, want.checksum);
        eq(tag + ' serverCount', ring.getServerCount(), want.serverCount);
        eq(tag + ' device serverCount', ring.deviceServerCount(), want.size / c.replicaPoints);
        eq(tag + ' servers', Object.keys(ring.servers), want.servers);
    });
    ring.destroy();
});
process.stdout.write(JSON.stringify({checks: checks, nfail: fails.length, fails: fails.slice(0, 20)}) + '\n');
