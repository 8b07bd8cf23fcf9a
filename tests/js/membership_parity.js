// membership_parity.js — replays tests/golden/membership_golden.json (what the reference's
// lib/membership did) through the drop-in membership module of ringpop-node_amd/js, installed
// the way a deployment installs it: into the module cache under <ringpopRoot>/lib/membership/
// index.js, then required through that path. Checks applied updates (rewritten values
// included), checksums, members arrays (join order), checksum strings and the events. Prints
// one JSON line.
'use strict';
var fs = require('fs');
var os = require('os');
var path = require('path');
var EventEmitter = require('events').EventEmitter;
var util = require('util');
var drop = require(path.join(__dirname, '..', '..', 'ringpop-node_amd', 'js', 'membership.js'));

var input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
// a stand-in ringpop checkout: the file must exist for require() to resolve it; install()
// makes the resolved path return the drop-in without running the file
var root = fs.mkdtempSync(path.join(os.tmpdir(), 'ringpop-'));
fs.mkdirSync(path.join(root, 'lib', 'membership'), {recursive: true});
fs.writeFileSync(path.join(root, 'lib', 'membership', 'index.js'), "throw new Error('not the drop-in');\n");
drop.install(root);
var initMembership = require(path.join(root, 'lib', 'membership', 'index.js'));
// every Member's 'dampScoreDecayed' in emission order, as ref_damp.js records the reference's
var decayed = [];
var origEmit = drop.Member.prototype.emit;
drop.Member.prototype.emit = function (ev, a, b) {
    if (ev === 'dampScoreDecayed') { decayed.push([this.address, a, b]); }
    return origEmit.apply(this, arguments);
};

var clock = 0;
Date.now = function () { return clock; };

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

var fails = [], checks = 0;
function eq(what, got, want) {
    checks++;
    if (JSON.stringify(got) !== JSON.stringify(want)) {
        fails.push({what: what, got: JSON.stringify(got).slice(0, 300), want: JSON.stringify(want).slice(0, 300)});
    }
}

input.cases.forEach(function (c) {
    var rp = new FakeRingpop(c.local);
    var m = initMembership(rp);
    rp.membership = m;
    eq(c.name + ' is the drop-in', m instanceof drop.Membership, true);
    var rands = c.joinRands, ri = 0;
    m.getJoinPosition = function () { return Math.floor((rands[ri++] / 4294967296) * this.members.length); };
    var ev = {updated: 0, set: 0, checksumComputed: 0, leave: 0};
    m.on('updated', function () { ev.updated++; });
    m.on('set', function () { ev.set++; });
    m.on('checksumComputed', function () { ev.checksumComputed++; });
    m.on('event', function (e) { if (e.name === 'localMemberLeave') { ev.leave++; } });
    var want = {updated: 0, set: 0};
    c.ops.forEach(function (op, j) {
        clock = op.now || 0;
        var tag = c.name + ' op ' + j;
        if (op.type === 'ready') {
            rp.isReady = op.value;
        } else if (op.type === 'set') {
            m.set();
            want.set++;
        } else {
            var changes = op.changes.map(function (ch, i) {
                return {address: ch[0], status: ch[1], incarnationNumber: ch[2], _i: i};
            });
            var applied = m.update(changes, op.isLocal);
            eq(tag + ' applied', applied.map(function (u) { return [u._i, u.status, u.incarnationNumber]; }),
                op.applied);
            if (op.applied.length) { want.updated++; }
        }
        eq(tag + ' checksum', m.checksum, op.checksum);
        if (op.members) {
            eq(tag + ' members', m.members.map(function (x) { return [x.address, x.status, x.incarnationNumber]; }),
                op.members);
        }
        if (typeof op.checksumString === 'string') { eq(tag + ' checksum string', m.generateChecksumString(), op.checksumString); }
    });
    eq(c.name + ' updated events', ev.updated, want.updated);
    eq(c.name + ' set events', ev.set, want.set);
    m.destroy();
});
// Damp scoring (tests/golden/damp_golden.json, the reference Membership / Member with damp
// scoring on): with dampScoringEnabled the drop-in keeps the scores on the device
// (rp_members_damp_*). Every member's dampScore, lastUpdateDampScore and lastUpdateTimestamp
// after every op, and the order of memberSuppressLimitExceeded events, must equal the
// reference's bit for bit.
function DampRingpop(whoami, cfgOver) {
    FakeRingpop.call(this, whoami);
    var conf = {
        dampScoringEnabled: true, dampScoringDecayEnabled: false, dampScoringDecayInterval: 1000,
        dampScoringHalfLife: 60, dampScoringInitial: 0, dampScoringMax: 10000, dampScoringMin: 0,
        dampScoringPenalty: 500, dampScoringReuseLimit: 2500, dampScoringSuppressLimit: 5000
    };
    Object.keys(cfgOver || {}).forEach(function (k) { conf[k] = cfgOver[k]; });
    this.config = {get: function (k) { return conf[k]; }};
}
util.inherits(DampRingpop, FakeRingpop);

(input.dampCases || []).forEach(function (c) {
    var rp = new DampRingpop(c.local, c.config);
    var m = initMembership(rp);
    rp.membership = m;
    m.getJoinPosition = function () { return this.members.length; };
    var suppressed = [];
    m.on('memberSuppressLimitExceeded', function (member) { suppressed.push(member.address); });
    c.ops.forEach(function (op, j) {
        clock = op.now;
        suppressed.length = 0;
        decayed.length = 0;
        var tag = 'damp ' + c.name + ' op ' + j, o = c.out[j];
        if (op.type === 'ready') {
            rp.isReady = op.value;
        } else if (op.type === 'set') {
            m.set();
        } else if (op.type === 'decay') {
            m._decayMembersDampScore();
        } else {
            var changes = op.changes.map(function (ch, i) {
                return {address: ch[0], status: ch[1], incarnationNumber: ch[2], _i: i};
            });
            var applied = m.update(changes, op.isLocal);
            eq(tag + ' applied', applied.map(function (u) { return u._i; }), o.applied);
        }
        eq(tag + ' suppressed', suppressed, o.suppressed);
        eq(tag + ' dampScoreDecayed', decayed, o.decayed);
        eq(tag + ' damp state', m.members.map(function (x) {
            return [x.address, x.dampScore, x.lastUpdateDampScore, x.lastUpdateTimestamp];
        }), o.members);
    });
    eq('damp ' + c.name + ' on the device', m._deviceDamp, !!rp.config.get('dampScoringEnabled'));
    m.destroy();
});

console.log(JSON.stringify({nfail: fails.length, checks: checks, fails: fails.slice(0, 20)}));
