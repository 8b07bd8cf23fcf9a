// ring_parity.js — replays tests/golden/ring_golden.json (what the reference's
// lib/ring/index.js returned) through the N-API HashRing of ringpop-node_amd/js and
// reports every mismatch. Driven by tests/test_js_gpu.py, which resolves the golden's
// UUID key recipes into explicit keys first (in.json). Prints one JSON line.
'use strict';
var fs = require('fs');
var path = require('path');
var amd = require(path.join(__dirname, '..', '..', 'ringpop-node_amd', 'js'));

var input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
var fails = [];
var checks = 0;

function makeHash(kind, mod) {  // tests/golden/ref_ring.js makeHash, with the engine's hash32
    if (kind === 'farmhash') { return null; }
    if (kind === 'port') {
        return function extractPort(s) { return parseInt(s.substr(s.lastIndexOf(':') + 1)); };
    }
    return function modHash(s) {
        if (s.charAt(0) === '#') { return parseInt(s.slice(1), 10); }
        return amd.hash32(s) % mod;
    };
}

function eq(what, got, want) {
    checks++;
    if (JSON.stringify(got) !== JSON.stringify(want)) {
        fails.push({what: what, got: String(JSON.stringify(got)).slice(0, 200), want: String(JSON.stringify(want)).slice(0, 200)});
    }
}

input.cases.forEach(function (c) {
    var opts = {replicaPoints: c.replicaPoints};
    var hf = makeHash(c.hashKind, c.hashMod);
    if (hf) { opts.hashFunc = hf; }
    var ring = new amd.HashRing(opts);
    var idx = {};
    c.names.forEach(function (n, i) { idx[n] = i; });
    function toIdx(x) { return x === null || x === undefined ? -1 : (x in idx ? idx[x] : 'unknown:' + x); }
    var events = {checksumComputed: 0};
    ring.on('checksumComputed', function () { events.checksumComputed++; });
    eq(c.name + ' initial checksum', ring.checksum, null);
    c.batches.forEach(function (b, bi) {
        var tag = c.name + '#' + bi;
        var before = events.checksumComputed;
        eq(tag + ' changed', ring.addRemoveServers(b.add, b.remove), b.changed);
        eq(tag + ' event', events.checksumComputed - before, b.changed ? 1 : 0);
        eq(tag + ' serverCount', ring.getServerCount(), b.serverCount);
        eq(tag + ' device serverCount', ring.deviceServerCount(), b.serverCount);
        eq(tag + ' servers (Object.keys order)', Object.keys(ring.servers), b.servers);
        eq(tag + ' getStats', ring.getStats(), {checksum: b.checksum, servers: b.servers});
        eq(tag + ' replicaPoints', ring.replicaPoints, c.replicaPoints);
        eq(tag + ' checksum', ring.checksum, b.checksum);
        if (!b.keys) { return; }
        eq(tag + ' lookup', ring.lookupBatch(b.keys).map(toIdx), b.lookup);
        Object.keys(b.lookupN).forEach(function (n) {
            var got = ring.lookupNBatch(b.keys, parseInt(n, 10)).map(function (row) { return row.map(toIdx); });
            eq(tag + ' lookupN ' + n, got, b.lookupN[n]);
        });
        // handleOrProxyAll's keysByDest = _.groupBy(keys, lookup) (index.js:616) and lookupKeys
        // (send.js:171-179), expected from the reference's recorded owners; JSON.stringify
        // keeps key order, so the first-seen dest order is checked too
        var want = {};
        b.keys.forEach(function (k, i) {
            var d = b.lookup[i] < 0 ? 'self:0' : c.names[b.lookup[i]];
            (want[d] = want[d] || []).push(k);
        });
        eq(tag + ' groupByOwner', ring.groupByOwner(b.keys, 'self:0'), want);
        eq(tag + ' groupBy (the documented handleOrProxyAll line)', ring.groupBy ? ring.groupBy(b.keys, 'self:0') : null, want);
        eq(tag + ' lookupKeys', ring.lookupKeys(b.keys, 'self:0'), Object.keys(want));
        // the single-key forms on a few keys
        for (var i = 0; i < Math.min(4, b.keys.length); i++) {
            eq(tag + ' lookup1', toIdx(ring.lookup(b.keys[i])), b.lookup[i]);
            if (b.lookupN['3']) { eq(tag + ' lookupN1', ring.lookupN(b.keys[i], 3).map(toIdx), b.lookupN['3'][i]); }
        }
    });
    // addServer / removeServer events (lib/ring/index.js:39-48,124-133)
    var added = [], removed = [];
    ring.on('added', function (n) { added.push(n); });
    ring.on('removed', function (n) { removed.push(n); });
    var probe = 'zz-probe:1';
    ring.addServer(probe);
    ring.addServer(probe);
    eq(c.name + ' hasServer', ring.hasServer(probe), true);
    ring.removeServer(probe);
    ring.removeServer(probe);
    eq(c.name + ' events', [added, removed], [[probe], [probe]]);
    eq(c.name + ' hasServer after remove', ring.hasServer(probe), false);
    ring.destroy();
});

process.stdout.write(JSON.stringify({checks: checks, fails: fails.slice(0, 20), nfail: fails.length}) + '\n');
