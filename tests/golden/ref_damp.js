// ref_damp.js — runs the REFERENCE Membership + Member (lib/membership/index.js, member.js from
// the reference checkout named on the command line) with damp scoring on, over the ops in
// <in.json>, and records every member's damp state after each op. Golden-vector generator only
// (tests/golden/make_damp_golden.py).
//
//   NODE_PATH=oracle/_ref/node_modules node tests/golden/ref_damp.js <ref_root> <in.json> <out.json>
//
// Injected: Date.now() (a virtual clock set per op), the config values of the case, and
// getJoinPosition (appends; the position does not touch damp state). Math.pow is wrapped to log
// every (exponent, result) pair the reference computes, so the restatement of the engine's pow
// can be checked bit for bit.
'use strict';
var fs = require('fs');
var path = require('path');
var EventEmitter = require('events').EventEmitter;
var util = require('util');

var refRoot = process.argv[2];
var input = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
var initMembership = require(path.join(refRoot, 'lib/membership/index.js'));
// every Member's 'dampScoreDecayed' (member.js:65), in emission order: [address, new, old]
var RefMember = require(path.join(refRoot, 'lib/membership/member.js'));
var decayed = [];
var origEmit = RefMember.prototype.emit;
RefMember.prototype.emit = function (ev, a, b) {
    if (ev === 'dampScoreDecayed') { decayed.push([this.address, a, b]); }
    return origEmit.apply(this, arguments);
};

var clock = 0;
Date.now = function () { return clock; };
var powLog = null;
var origPow = Math.pow;
Math.pow = function (a, b) {
    var r = origPow(a, b);
    if (powLog && a === Math.E) { powLog.push([b, r]); }
    return r;
};

function FakeRingpop(whoami, cfg) {
    EventEmitter.call(this);
    this.hostPort = whoami;
    this.isReady = true;
    this.logger = {debug: function () {}, info: function () {}, warn: function () {}, error: function () {}};
    var conf = {
        dampScoringEnabled: true, dampScoringDecayEnabled: false, dampScoringDecayInterval: 1000,
        dampScoringHalfLife: 60, dampScoringInitial: 0, dampScoringMax: 10000, dampScoringMin: 0,
        dampScoringPenalty: 500, dampScoringReuseLimit: 2500, dampScoringSuppressLimit: 5000
    };
    Object.keys(cfg || {}).forEach(function (k) { conf[k] = cfg[k]; });
    this.config = {get: function (k) { return conf[k]; }};
}
util.inherits(FakeRingpop, EventEmitter);
FakeRingpop.prototype.whoami = function () { return this.hostPort; };
FakeRingpop.prototype.stat = function () {};

var out = {node: process.version, cases: []};
input.cases.forEach(function (c) {
    var rp = new FakeRingpop(c.local, c.config);
    var m = initMembership(rp);
    rp.membership = m;
    m.getJoinPosition = function () { return this.members.length; };
    var suppressed = [];
    m.on('memberSuppressLimitExceeded', function (member) { suppressed.push(member.address); });
    var co = {name: c.name, ops: []};
    c.ops.forEach(function (op) {
        clock = op.now;
        powLog = [];
        suppressed.length = 0;
        decayed.length = 0;
        var o = {};
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
            o.applied = applied.map(function (u) { return u._i; });
        }
        o.suppressed = suppressed.slice();
        o.decayed = decayed.slice();
        o.members = m.members.map(function (x) {
            return [x.address, x.dampScore, x.lastUpdateDampScore, x.lastUpdateTimestamp];
        });
        o.pow = powLog;
        co.ops.push(o);
    });
    powLog = null;
    out.cases.push(co);
});
fs.writeFileSync(process.argv[4], JSON.stringify(out));
