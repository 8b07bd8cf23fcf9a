// ref_sim.js — drives the REFERENCE ringpop modules of N in-process nodes through the
// deterministic gossip round model (oracle/orc_sim.c header; DESIGN.md §SWIM round model) and
// records every live node's membership checksum after each round. Golden-vector generator
// only (tests/golden/make_golden.py); never shipped, never run on the GPU box.
//
//   NODE_PATH=oracle/_ref/node_modules node tests/golden/ref_sim.js <ref_root> <in.json> <out.json>
//
// Scenario events (c.events = [[round, kind, node], ...], applied before that round's phase A):
// 'kill' (the node stops: crash / SIGSTOP, scripts/tick-cluster.js:417-470), 'revive' (SIGCONT:
// back with its state intact), 'leave' (the admin leave handler, server/admin/member.js:70-98:
// makeLeave(whoami, localMember.incarnationNumber), as benchmarks/convergence-time/scenarios/
// send it), 'join' (a fresh process for the node bootstraps into the running cluster, index.js:
// 240-322: makeAlive(self, Date.now()); three live nodes chosen by the JOIN Philox stream answer
// the join (server/protocol/join.js:126-133: makeAlive(joiner, its incarnation), then
// {checksum, membership: fullSync()}); mergeJoinResponses (join-sender.js:253-256,
// join-response-merge.js:40-56) -> update (stashed) -> set() -> the set handler
// (on_membership_event.js:42-67) -> ready; the model clears the dissemination as at
// bootstrap; gossip.start shuffles).
//
// Reference code doing the work per node: lib/membership (Membership, Member, merge),
// lib/gossip/dissemination.js, lib/gossip/suspicion.js, lib/membership/iterator.js,
// lib/ring (HashRing, only for maxPiggybackCount), lib/on_membership_event.js (wiring).
// The harness replaces only transport and time: TChannel ping/ping-req become synchronous
// calls in the model's phase order (restating ping-sender.js / ping-req-sender.js /
// server/protocol/ping*.js), setTimeout is a round-based virtual timer, Date.now() is
// now0 + 200*round, and Math.random-driven shuffle/sample are the Philox streams SHUF/SAMP.
'use strict';
var fs = require('fs');
var path = require('path');
var EventEmitter = require('events').EventEmitter;
var util = require('util');

var refRoot = process.argv[2];
var input = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
var R = function (p) { return require(path.join(refRoot, p)); };

// ---- Philox4x32-10 (must equal oracle/orc_philox.c; checked below against Random123)
function mulhilo(a, b) {
    var al = a & 0xffff, ah = a >>> 16, bl = b & 0xffff, bh = b >>> 16;
    var t = al * bl;
    var u = ah * bl + (t >>> 16);
    var v = al * bh + (u % 65536);
    var hi = ah * bh + Math.floor(u / 65536) + Math.floor(v / 65536);
    return [hi >>> 0, Math.imul(a, b) >>> 0];
}
function philox(c, k) {
    var c0 = c[0] >>> 0, c1 = c[1] >>> 0, c2 = c[2] >>> 0, c3 = c[3] >>> 0, k0 = k[0] >>> 0, k1 = k[1] >>> 0;
    for (var r = 0; r < 10; r++) {
        var p0 = mulhilo(0xD2511F53, c0), p1 = mulhilo(0xCD9E8D57, c2);
        var n0 = (p1[0] ^ c1 ^ k0) >>> 0, n1 = p1[1], n2 = (p0[0] ^ c3 ^ k1) >>> 0, n3 = p0[1];
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 = (k0 + 0x9E3779B9) >>> 0; k1 = (k1 + 0xBB67AE85) >>> 0;
    }
    return [c0, c1, c2, c3];
}
(function kat() {
    var r = philox([0, 0, 0, 0], [0, 0]);
    if (r[0] !== 0x6627e8d5 || r[3] !== 0x9b00dbd8) { throw new Error('philox KAT failed'); }
})();
var TAG_SHUF = 0x53485546, TAG_SAMP = 0x53414d50, TAG_JOIN = 0x4a4f494e;
function scaled(r, n) { return Math.floor((r / 4294967296) * n); }  // == (r*n)>>32 for n < 2^21

// ---- virtual time
var round = 0, now0 = 0, suspRounds = 25, seq = 0;
Date.now = function () { return now0 + 200 * round; };
global.setTimeout = function (fn) { return {fn: fn, due: round + suspRounds, seq: seq++, cancelled: false, fired: false}; };
global.clearTimeout = function (h) { if (h) { h.cancelled = true; } };

var initMembership = R('lib/membership/index.js');
var Dissemination = R('lib/gossip/dissemination.js');
var Suspicion = R('lib/gossip/suspicion.js');
var MembershipIterator = R('lib/membership/iterator.js');
var HashRing = R('lib/ring/index.js');
var onMembershipEvent = R('lib/on_membership_event.js');
var mergeJoinResponses = R('lib/gossip/join-response-merge.js');

function FakeRingpop(whoami) {
    EventEmitter.call(this);
    this.hostPort = whoami;
    this.isReady = false;
    this.logger = {debug: function () {}, info: function () {}, warn: function () {}, error: function () {}};
    this.config = {get: function (k) {
        return {dampScoringEnabled: false, dampScoringDecayEnabled: false, dampScoringInitial: 0}[k];
    }};
    this.membershipUpdateRollup = {trackUpdates: function () {}};
    this.fullSyncs = 0;
}
util.inherits(FakeRingpop, EventEmitter);
FakeRingpop.prototype.whoami = function () { return this.hostPort; };
FakeRingpop.prototype.stat = function (type, key) { if (key === 'full-sync') { this.fullSyncs++; } };

function digits(n) { var d = 0; while (n) { d++; n = Math.floor(n / 10); } return d; }
function wire(x) { return JSON.parse(JSON.stringify(x)); }

var out = {cases: []};
input.cases.forEach(function (c) {
    var N = c.names.length, seed = c.seed;
    now0 = c.now0; suspRounds = c.suspRounds; round = 0;
    var idOf = {};
    c.names.forEach(function (a, i) { idOf[a] = i; });
    var dead = c.dead;
    function makeNode(addr, v) {
        var rp = new FakeRingpop(addr);
        rp.ring = new HashRing({replicaPoints: 1});
        rp.membership = initMembership(rp);
        rp.dissemination = new Dissemination(rp);
        rp.suspicion = new Suspicion({ringpop: rp, suspicionTimeout: 5000});
        rp.memberIterator = new MembershipIterator(rp);
        // the protocol-period loop is the harness's phase A; a local leave stops it
        // (LocalMemberLeaveEvent -> gossip.stop(), on_membership_event.js:32-40)
        rp.gossip = {isStopped: false, stop: function () { this.isStopped = true; }};
        onMembershipEvent.register(rp);
        var m = rp.membership;
        var nsh = 0;
        m.shuffle = function () {  // _.shuffle -> Fisher-Yates over SHUF(shuffle#, i, v)
            var a = this.members.slice();
            var s = nsh++;
            for (var i = a.length - 1; i >= 1; i--) {
                var j = scaled(philox([s, i, v, 0], [seed, TAG_SHUF])[0], i + 1);
                var t = a[i]; a[i] = a[j]; a[j] = t;
            }
            this.members = a;
        };
        m.getRandomPingableMembers = function (n, excluding) {  // _.sample -> partial FY over SAMP(round, i, v)
            var self = this;
            var cands = this.members.filter(function (x) {
                return excluding.indexOf(x.address) < 0 && self.isPingable(x);
            });
            var k = Math.min(n, cands.length);
            for (var i = 0; i < k; i++) {
                var j = i + scaled(philox([round, i, v, 0], [seed, TAG_SAMP])[0], cands.length - i);
                var t = cands[i]; cands[i] = cands[j]; cands[j] = t;
            }
            return cands.slice(0, k);
        };
        return rp;
    }
    var nodes = c.names.map(function (addr, v) {
        var rp = makeNode(addr, v);
        var m = rp.membership;
        // bootstrap (index.js:270-322): self alive, stash the rest, set(), ready
        m.makeAlive(addr, c.inc0[v]);
        m.update(c.names.map(function (a, i) {
            return {address: a, status: 'alive', incarnationNumber: c.inc0[i]};
        }).filter(function (u) { return u.address !== addr; }));
        m.set();
        rp.isReady = true;
        rp.dissemination.clearChanges();
        rp.dissemination.maxPiggybackCount = 15 * digits(N);
        if (!dead[v]) { m.shuffle(); }  // gossip.start (gossip/index.js:97)
        return rp;
    });
    var down = dead.slice();
    function live(v) { return !down[v]; }
    var co = {name: c.name, rounds: [], maxPiggyback: []};
    for (round = 0; round < c.rounds; round++) {
        (c.events || []).forEach(function (e) {
            if (e[0] !== round) { return; }
            var v = e[2];
            if (e[1] === 'kill') { down[v] = 1; }
            if (e[1] === 'revive') { down[v] = 0; }
            if (e[1] === 'join') {
                var addr = c.names[v], incv = Date.now();
                var prev = nodes[v];
                var rp = makeNode(addr, v);
                rp.fullSyncs = prev.fullSyncs;
                rp.membership.makeAlive(addr, incv);
                // the responders: 3 live nodes other than v, partial Fisher-Yates over them in id
                // order with the JOIN stream (join-sender.js selects from the bootstrap hosts)
                var cands = [];
                for (var u = 0; u < N; u++) { if (u !== v && live(u)) { cands.push(u); } }
                var nj = Math.min(3, cands.length);
                for (var q = 0; q < nj; q++) {
                    var jj = q + scaled(philox([round, q, v, 0], [seed, TAG_JOIN])[0], cands.length - q);
                    var tt = cands[q]; cands[q] = cands[jj]; cands[jj] = tt;
                }
                var responses = cands.slice(0, nj).map(function (u) {
                    nodes[u].membership.makeAlive(addr, incv);  // join.js:126
                    return wire({checksum: nodes[u].membership.checksum,
                        members: nodes[u].dissemination.fullSync()});
                });
                rp.membership.update(mergeJoinResponses(rp, responses));  // stashed: not ready
                rp.membership.set();
                rp.isReady = true;
                rp.dissemination.clearChanges();
                rp.membership.shuffle();  // gossip.start
                nodes[v] = rp;
                down[v] = 0;
            }
            if (e[1] === 'leave') {  // server/admin/member.js:76-93, while the node is up
                var lm = nodes[v].membership.localMember;
                if (live(v) && lm.status !== 'leave') {
                    nodes[v].membership.makeLeave(c.names[v], lm.incarnationNumber);
                }
            }
        });
        var target = [], ping = [], resp = [];
        // A
        for (var v = 0; v < N; v++) {
            target[v] = -1;
            if (!live(v) || nodes[v].gossip.isStopped) { continue; }
            var t = nodes[v].memberIterator.next();
            if (!t) { continue; }
            target[v] = idOf[t.address];
            var m = nodes[v].membership;
            ping[v] = wire({checksum: m.checksum, changes: nodes[v].dissemination.issueAsSender(),
                source: c.names[v], sourceIncarnationNumber: m.getIncarnationNumber()});
        }
        // B
        for (v = 0; v < N; v++) {
            var j = target[v];
            if (j < 0 || !live(j)) { continue; }
            nodes[j].membership.update(ping[v].changes);
            resp[v] = wire({changes: nodes[j].dissemination.issueAsReceiver(ping[v].source,
                ping[v].sourceIncarnationNumber, ping[v].checksum)});
        }
        // C
        for (v = 0; v < N; v++) {
            j = target[v];
            if (j < 0 || !live(j)) { continue; }
            nodes[v].membership.update(resp[v].changes);
            nodes[v].membership.update(resp[v].changes);
        }
        // D1
        var helpers = [], legs = [];
        for (v = 0; v < N; v++) {
            j = target[v];
            helpers[v] = [];
            if (j < 0 || live(j)) { continue; }
            m = nodes[v].membership;
            var tm = m.findMemberByAddress(c.names[j]);
            var hs = m.getRandomPingableMembers(3, [tm.address]);
            if (hs.length === 0) { m.makeSuspect(tm.address, tm.incarnationNumber); continue; }
            helpers[v] = hs.map(function (x) { return idOf[x.address]; });
            legs[v] = hs.map(function () {
                return wire({checksum: m.checksum, changes: nodes[v].dissemination.issueAsSender(),
                    source: c.names[v], sourceIncarnationNumber: m.getIncarnationNumber(), target: c.names[j]});
            });
        }
        // D2
        var lresp = [];
        for (v = 0; v < N; v++) {
            lresp[v] = [];
            for (var k = 0; k < helpers[v].length; k++) {
                var h = helpers[v][k];
                if (!live(h)) { lresp[v][k] = null; continue; }
                var body = legs[v][k];
                nodes[h].membership.update(body.changes);
                nodes[h].dissemination.issueAsSender();  // the helper's own ping of the dead target
                lresp[v][k] = wire({changes: nodes[h].dissemination.issueAsReceiver(body.source,
                    body.sourceIncarnationNumber, body.checksum), pingStatus: false, target: body.target});
            }
        }
        // D3
        for (v = 0; v < N; v++) {
            if (!helpers[v].length) { continue; }
            var bad = false;
            for (k = 0; k < helpers[v].length; k++) {
                if (!lresp[v][k]) { continue; }
                nodes[v].membership.update(lresp[v][k].changes);
                bad = true;
            }
            if (bad) {
                tm = nodes[v].membership.findMemberByAddress(c.names[target[v]]);
                nodes[v].membership.makeSuspect(tm.address, tm.incarnationNumber);
            }
        }
        // E
        for (v = 0; v < N; v++) {
            if (!live(v)) { continue; }
            var timers = nodes[v].suspicion.timers;
            var due = Object.keys(timers).filter(function (a) {
                var x = timers[a];
                return x && !x.cancelled && !x.fired && x.due <= round;
            }).sort(function (a, b) { return idOf[a] - idOf[b]; });
            due.forEach(function (a) { var x = timers[a]; x.fired = true; x.fn(); });
        }
        var cks = [];
        for (v = 0; v < N; v++) { cks.push(live(v) ? nodes[v].membership.checksum : 0); }
        co.rounds.push(cks);
        co.maxPiggyback.push(nodes.map(function (x) { return x.dissemination.maxPiggybackCount; }));
    }
    co.fullSyncs = nodes.reduce(function (a, x) { return a + x.fullSyncs; }, 0);
    co.finalViews = (c.views || []).map(function (v) {
        return nodes[v].membership.members.map(function (x) { return [x.address, x.status, x.incarnationNumber]; });
    });
    out.cases.push(co);
});
fs.writeFileSync(process.argv[4], JSON.stringify(out));
