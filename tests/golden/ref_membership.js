// ref_membership.js — runs the REFERENCE Membership (lib/membership/index.js, member.js,
// merge.js from the reference checkout given on the command line) over the ops in <in.json>
// and records what it did. Golden-vector generator only (tests/golden/make_golden.py).
//
//   NODE_PATH=oracle/_ref/node_modules node tests/golden/ref_membership.js <ref_root> <in.json> <out.json>
//
// Injected (never random): Date.now() (virtual clock per op), getJoinPosition (Math.random
// replaced by the u32 stream in the case: floor(r / 2^32 * members.length)). `farmhash` is the
// oracle's N-API restatement; underscore/node-uuid are the minimal stand-ins of oracle/gen/shims.
'use strict';
var fs = require('fs');
var path = require('path');
var EventEmitter = require('events').EventEmitter;
var util = require('util');

var refRoot = process.argv[2];
var input = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
var initMembership = require(path.join(refRoot, 'lib/membership/index.js'));

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

function snapshot(m) {
    return m.members.map(function (x) { return [x.address, x.status, x.incarnationNumber]; });
}

var out = {cases: []};
input.cases.forEach(function (c) {
    var rp = new FakeRingpop(c.local);
    var m = initMembership(rp);
    rp.membership = m;
    var rands = c.joinRands || [];
    var ri = 0;
    m.getJoinPosition = function () {
        var r = rands[ri++];
        if (r === undefined) { throw new Error('join stream exhausted'); }
        return Math.floor((r / 4294967296) * this.members.length);
    };
    var co = {name: c.name, ops: []};
    c.ops.forEach(function (op) {
        clock = op.now || 0;
        var o = {};
        if (op.type === 'ready') {
            rp.isReady = op.value;
        } else if (op.type === 'set') {
            m.set();
        } else {
            var changes = op.changes.map(function (ch, i) {
                return {address: ch[0], status: ch[1], incarnationNumber: ch[2], _i: i};
            });
            var applied = m.update(changes, op.isLocal);
            o.applied = applied.map(function (u) { return [u._i, u.status, u.incarnationNumber]; });
        }
        o.checksum = m.checksum;
        if (op.members) { o.members = snapshot(m); }
        if (op.checksumString) { o.checksumString = m.generateChecksumString(); }
        co.ops.push(o);
    });
    out.cases.push(co);
});
fs.writeFileSync(process.argv[4], JSON.stringify(out));
