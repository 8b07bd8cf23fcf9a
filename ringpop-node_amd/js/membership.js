// membership.js — a drop-in for ringpop's lib/membership/index.js (initMembership) whose
// update / set / checksum run on the MI355X engine (rp_members_* through rpamd.node).
//
// The reference builds its membership with `initMembership(this)` (index.js:137), required
// relatively (index.js:51), so it is not injectable through options. install(ringpopRoot)
// seeds Node's module cache for that file, so the reference's own require returns this module:
//
//     require('ringpop-node_amd/js/membership').install(path.dirname(require.resolve('ringpop')));
//     var RingPop = require('ringpop');   // index.js now gets the device-backed membership
//
// Everything the rest of ringpop reads stays a plain JS object, kept coherent with the device
// table after every call: `members` (join order, getJoinPosition), `membersByAddress`,
// `localMember`, `checksum`, `stashedUpdates`, Member objects (EventEmitters with address /
// status / incarnationNumber / dampScore) and the events 'updated', 'set', 'checksumComputed',
// 'checksumUpdate', 'event' (LocalMemberLeaveEvent), 'memberSuppressLimitExceeded'. The
// override rules (member.js:71-202), the order-sensitive fold (index.js:272-304), the
// stash merge (merge.js:22-51) and the checksum (index.js:48-123) are the device's.
'use strict';
var crypto = require('crypto');
var EventEmitter = require('events').EventEmitter;
var Module = require('module');
var path = require('path');
var util = require('util');

var amd = require('./index.js');
var native = amd.native;

var STATUS = amd.STATUS;
var STATUS_CODE = {alive: 0, suspect: 1, faulty: 2, leave: 3};
var Status = {alive: 'alive', faulty: 'faulty', leave: 'leave', suspect: 'suspect'};

function cfg(ringpop, key, dflt) {
    var v = ringpop.config && typeof ringpop.config.get === 'function' ? ringpop.config.get(key) : undefined;
    return v === undefined || v === null ? dflt : v;
}

function uuidV4() {
    var b = crypto.randomBytes(16);
    b[6] = (b[6] & 0x0f) | 0x40;
    b[8] = (b[8] & 0x3f) | 0x80;
    var h = b.toString('hex');
    return h.slice(0, 8) + '-' + h.slice(8, 12) + '-' + h.slice(12, 16) + '-' + h.slice(16, 20) + '-' + h.slice(20);
}

// new Update(address, inc, status, localMember) — lib/membership/update.js:26-42
function makeUpdate(address, incarnationNumber, status, localMember) {
    localMember = localMember || {};
    return {
        id: uuidV4(), address: address, incarnationNumber: incarnationNumber, status: status,
        source: localMember.address, sourceIncarnationNumber: localMember.incarnationNumber, timestamp: Date.now()
    };
}

// LocalMemberLeaveEvent — lib/membership/events.js
function LocalMemberLeaveEvent(member, oldStatus) {
    this.name = LocalMemberLeaveEvent.Name;
    this.member = member;
    this.oldStatus = oldStatus;
}
LocalMemberLeaveEvent.Name = 'localMemberLeave';

// Member (lib/membership/member.js:28-41): the JS object the rest of ringpop holds. Its state
// is written from the device's verdicts. With dampScoringEnabled the damp scores are the
// device's too (rp_members_damp_*: the penalty folded with each update batch, the decayer
// sweep); otherwise only lastUpdateTimestamp moves, as in the reference.
function Member(ringpop, update) {
    EventEmitter.call(this);
    this.ringpop = ringpop;
    this.id = update.address;
    this.address = update.address;
    this.status = update.status;
    this.incarnationNumber = update.incarnationNumber;
    var ds = update.dampScore;
    this.dampScore = typeof ds === 'number' && !isNaN(ds) ? ds : cfg(ringpop, 'dampScoringInitial', 0);
    this.dampedTimestamp = update.dampedTimestamp;
    this.lastUpdateTimestamp = null;
    this.lastUpdateDampScore = this.dampScore;
    this.Date = Date;
}
util.inherits(Member, EventEmitter);
Member.Status = Status;

// score(t2) = score(t1) * e^(-(t2 - t1) ln2 / halfLife), rounded, >= dampScoringMin (member.js:45-66)
Member.prototype.decayDampScore = function decayDampScore() {
    if (this.dampScore === null || this.dampScore === undefined) {
        this.dampScore = cfg(this.ringpop, 'dampScoringInitial', 0);
        return;
    }
    var secs = (this.Date.now() - this.lastUpdateTimestamp) / 1000;
    var decay = Math.pow(Math.E, -1 * secs * Math.LN2 / cfg(this.ringpop, 'dampScoringHalfLife', 60));
    var old = this.dampScore;
    this.dampScore = Math.max(Math.round(this.lastUpdateDampScore * decay), cfg(this.ringpop, 'dampScoringMin', 0));
    this.emit('dampScoreDecayed', this.dampScore, old);
};

Member.prototype._applyUpdatePenalty = function _applyUpdatePenalty() {  // member.js:133-153
    this.decayDampScore();
    this.dampScore = Math.min(this.dampScore + cfg(this.ringpop, 'dampScoringPenalty', 500),
        cfg(this.ringpop, 'dampScoringMax', 10000));
    if (this.dampScore > cfg(this.ringpop, 'dampScoringSuppressLimit', 5000)) { this.emit('suppressLimitExceeded'); }
};

Member.prototype.getStats = function getStats() {
    return {address: this.address, status: this.status, incarnationNumber: this.incarnationNumber,
        dampScore: this.dampScore};
};

// The device's verdict on an existing member, applied the way evaluateUpdate does after its
// rules passed (member.js:86-121): status (a local leave emits LocalMemberLeaveEvent),
// incarnation, damp penalty, 'updated'. damp (device damp scoring): {score, exceeded, now} of
// this change from rp_members_damp_last — the score after _applyUpdatePenalty and whether it
// passed the suppress limit.
Member.prototype._applyVerdict = function _applyVerdict(update, damp) {
    var oldStatus = this.status;
    if (this.status !== update.status) {
        this.status = update.status;
        if (this.address === this.ringpop.whoami() && this.status === Status.leave) {
            this.ringpop.membership.emit('event', new LocalMemberLeaveEvent(this, oldStatus));
        }
    }
    if (this.incarnationNumber !== update.incarnationNumber) { this.incarnationNumber = update.incarnationNumber; }
    if (cfg(this.ringpop, 'dampScoringEnabled', false) && update.address !== this.ringpop.whoami()) {
        if (damp) {
            // _applyUpdatePenalty starts with decayDampScore, which emits 'dampScoreDecayed'
            // (decayed, previous) before the penalty (member.js:45-66,136): the decayed value is
            // the same expression over this member's last score and timestamp at the device's now
            var old = this.dampScore;
            if (old !== null && old !== undefined) {
                var decay = Math.pow(Math.E, -1 * ((damp.now - this.lastUpdateTimestamp) / 1000) * Math.LN2 /
                    cfg(this.ringpop, 'dampScoringHalfLife', 60));
                this.emit('dampScoreDecayed', Math.max(Math.round(this.lastUpdateDampScore * decay),
                    cfg(this.ringpop, 'dampScoringMin', 0)), old);
            }
            this.dampScore = damp.score;
            if (damp.exceeded) { this.emit('suppressLimitExceeded'); }
        } else {
            this._applyUpdatePenalty();
        }
        this.lastUpdateDampScore = this.dampScore;
    }
    this.emit('updated', update);
    this.lastUpdateTimestamp = damp ? damp.now : this.Date.now();
};

// Membership (lib/membership/index.js:34-46) over one rp_members handle.
function Membership(opts) {
    EventEmitter.call(this);
    this.ringpop = opts.ringpop;
    this.setTimeout = opts.setTimeout || setTimeout;
    this.clearTimeout = opts.clearTimeout || clearTimeout;
    this.members = [];
    this.membersByAddress = {};
    this.checksum = null;
    this.stashedUpdates = [];
    this.decayTimer = null;
    this.device = opts.device || 0;
    if (native.deviceCount() <= this.device) {
        throw new Error('ringpop_amd: no HIP device ' + this.device + ' for the membership engine');
    }
    this._h = native.membersCreate(opts.capacity || 1024, this.device);
    this._ids = {};  // address -> interned id
    this._local = null;
    // damp scoring on the device when the config enables it (decided at the first call that
    // needs it: initMembership's ringpop has its config by then)
    this._deviceDamp = null;
}
util.inherits(Membership, EventEmitter);

Membership.prototype._intern = function _intern(addresses) {
    var ids = new Uint32Array(addresses.length), miss = [], where = [];
    for (var i = 0; i < addresses.length; i++) {
        var id = this._ids[addresses[i]];
        if (id === undefined) {
            miss.push(addresses[i]);
            where.push(i);
        } else {
            ids[i] = id;
        }
    }
    if (miss.length) {
        var got = native.membersIntern(this._h, miss);
        for (var j = 0; j < miss.length; j++) {
            this._ids[miss[j]] = got[j];
            ids[where[j]] = got[j];
        }
    }
    var me = this.ringpop.whoami();
    if (this._local !== me) {
        this._local = me;
        native.membersSetLocal(this._h, this._intern([me])[0]);
    }
    return ids;
};

// Whether damp scores live on the device; the first call configures rp_members_damp_* from
// ringpop's config (config.js:60-71 names and defaults).
Membership.prototype._damp = function _damp() {
    if (this._deviceDamp === null) {
        this._deviceDamp = !!cfg(this.ringpop, 'dampScoringEnabled', false);
        if (this._deviceDamp) {
            native.membersDampConfigure(this._h, {
                enabled: true,
                initial: cfg(this.ringpop, 'dampScoringInitial', 0),
                min: cfg(this.ringpop, 'dampScoringMin', 0),
                max: cfg(this.ringpop, 'dampScoringMax', 10000),
                penalty: cfg(this.ringpop, 'dampScoringPenalty', 500),
                suppressLimit: cfg(this.ringpop, 'dampScoringSuppressLimit', 5000),
                halfLife: cfg(this.ringpop, 'dampScoringHalfLife', 60)
            });
        }
    }
    return this._deviceDamp;
};

Membership.prototype._columns = function _columns(changes) {
    var k = changes.length, st = new Uint8Array(k), inc = new Float64Array(k), addr = new Array(k);
    for (var i = 0; i < k; i++) {
        var code = STATUS_CODE[changes[i].status];
        if (code === undefined) { throw new Error('ringpop_amd: unknown member status ' + changes[i].status); }
        addr[i] = changes[i].address;
        st[i] = code;
        inc[i] = changes[i].incarnationNumber;
    }
    return {ids: this._intern(addr), st: st, inc: inc};
};

// computeChecksum (index.js:48-75): the device hashes the address-sorted checksum string
Membership.prototype.computeChecksum = function computeChecksum() {
    return this._takeChecksum(native.membersComputeChecksum);
};

// The checksum `read` returns, taken with computeChecksum's events and stats. update() passes
// the read of the checksum its batch already built on the device (rp_members_update computes
// it once per applied batch, index.js:306-309), so a batch hashes its string once.
Membership.prototype._takeChecksum = function _takeChecksum(read) {
    var start = new Date();
    var prev = this.checksum;
    this.checksum = read(this._h);
    this.emit('checksumComputed');
    this.ringpop.stat('timing', 'compute-checksum', start);
    this.ringpop.stat('gauge', 'checksum', this.checksum);
    if (prev !== this.checksum) { this._emitChecksumUpdate(); }
    return this.checksum;
};

Membership.prototype._emitChecksumUpdate = function _emitChecksumUpdate() {  // index.js:77-94
    var counts = {alive: 0, faulty: 0, leave: 0, suspect: 0};
    for (var i = 0; i < this.members.length; i++) { counts[this.members[i].status] += 1; }
    this.emit('checksumUpdate', {local: this.ringpop.whoami(), timestamp: Date.now(), checksum: this.checksum,
        membershipStatusCounts: counts});
};

Membership.prototype.findMemberByAddress = function findMemberByAddress(address) {
    return this.membersByAddress[address];
};

// generateChecksumString (index.js:100-123), built on the device
Membership.prototype.generateChecksumString = function generateChecksumString() {
    return this.members.length ? native.membersChecksumString(this._h) : '';
};

Membership.prototype.getIncarnationNumber = function getIncarnationNumber() {
    return this.localMember && this.localMember.incarnationNumber;
};

Membership.prototype.getJoinPosition = function getJoinPosition() {  // index.js:129-131
    return Math.floor(Math.random() * this.members.length);
};

Membership.prototype.getMemberAt = function getMemberAt(index) { return this.members[index]; };
Membership.prototype.getMemberCount = function getMemberCount() { return this.members.length; };

// _.sample(pingable members not excluded, n) (index.js:141-150)
Membership.prototype.getRandomPingableMembers = function getRandomPingableMembers(n, excluding) {
    var self = this;
    var c = this.members.filter(function (m) { return excluding.indexOf(m.address) < 0 && self.isPingable(m); });
    var k = Math.min(Math.max(n, 0), c.length);
    for (var i = 0; i < k; i++) {
        var j = i + Math.floor(Math.random() * (c.length - i));
        var t = c[i]; c[i] = c[j]; c[j] = t;
    }
    return c.slice(0, k);
};

Membership.prototype.getStats = function getStats() {
    return {checksum: this.checksum, members: this.members.map(function (m) { return m.getStats(); })
        .sort(function (a, b) { return a.address.localeCompare(b.address); })};
};

Membership.prototype.hasMember = function hasMember(member) { return !!this.findMemberByAddress(member.address); };

Membership.prototype.isPingable = function isPingable(member) {  // index.js:173-177
    return member.address !== this.ringpop.whoami() &&
        (member.status === Status.alive || member.status === Status.suspect);
};

Membership.prototype.makeAlive = function makeAlive(address, incarnationNumber) {
    this.ringpop.stat('increment', 'make-alive');
    return this._updateMember(makeUpdate(address, incarnationNumber, Status.alive, this.localMember),
        address === this.ringpop.whoami());
};
Membership.prototype.makeFaulty = function makeFaulty(address, incarnationNumber) {
    this.ringpop.stat('increment', 'make-faulty');
    return this._updateMember(makeUpdate(address, incarnationNumber, Status.faulty, this.localMember));
};
Membership.prototype.makeLeave = function makeLeave(address, incarnationNumber) {
    this.ringpop.stat('increment', 'make-leave');
    return this._updateMember(makeUpdate(address, incarnationNumber, Status.leave, this.localMember));
};
Membership.prototype.makeSuspect = function makeSuspect(address, incarnationNumber) {
    this.ringpop.stat('increment', 'make-suspect');
    return this._updateMember(makeUpdate(address, incarnationNumber, Status.suspect, this.localMember));
};

// Membership.set (index.js:208-247): the stash is merged on the device (merge.js:22-51), the
// picked changes become Member objects appended in first-seen order, checksum once, 'set'.
Membership.prototype.set = function set() {
    if (this.ringpop.isReady || this.stashedUpdates === null) { return; }
    if (!Array.isArray(this.stashedUpdates) || this.stashedUpdates.length === 0) { return; }
    var stash = [];
    this.stashedUpdates.forEach(function (batch) { for (var i = 0; i < batch.length; i++) { stash.push(batch[i]); } });
    var col = this._columns(stash);
    var pick = native.membersSet(this._h, col.ids, col.st, col.inc);
    var updates = [];
    for (var i = 0; i < pick.length; i++) {
        var update = stash[pick[i]];
        var member = this._createMember(update);
        this.members.push(member);
        this.membersByAddress[member.address] = member;
        updates.push(update);
    }
    this.stashedUpdates = null;
    this.computeChecksum();
    this.emit('set', updates);
};

// Membership.update (index.js:249-324): the batch is folded on the device (override rules,
// local override with Date.now(), in array order per address); the verdicts are mirrored into
// the Member objects in batch order, then one checksum and 'updated'.
Membership.prototype.update = function update(changes, isLocal) {
    changes = Array.isArray(changes) ? changes : [changes];
    this.ringpop.stat('gauge', 'changes.apply', changes.length);
    if (changes.length === 0) { return []; }
    if (!isLocal && !this.ringpop.isReady) {  // buffer until ready (259-265)
        if (Array.isArray(this.stashedUpdates)) { this.stashedUpdates.push(changes); }
        return [];
    }
    var col = this._columns(changes);
    var deviceDamp = this._damp();
    var now = Date.now();
    var r = native.membersUpdate(this._h, col.ids, col.st, col.inc, now);
    var d = deviceDamp && r.nApplied > 0 ? native.membersDampLast(this._h, changes.length) : null;
    var updates = [];
    for (var i = 0; i < changes.length; i++) {
        var a = r.applied[i];
        if (!a) { continue; }
        var change = changes[i];
        if (a === 2) {  // an unknown address: created verbatim at a random join position (277-293)
            var member = this._createMember(change);
            if (member.address === this.ringpop.whoami()) { this.localMember = member; }
            this.members.splice(this.getJoinPosition(), 0, member);
            this.membersByAddress[member.address] = member;
            updates.push(change);
            continue;
        }
        var st = STATUS[r.status[i]], inc = r.inc[i];
        var upd = change;
        if (st !== change.status || inc !== change.incarnationNumber) {  // the local override's rewrite
            upd = {status: st, incarnationNumber: inc};
            for (var key in change) { if (!(key in upd)) { upd[key] = change[key]; } }
        }
        this.membersByAddress[change.address]._applyVerdict(upd,
            d ? {score: d.score[i], exceeded: d.exceeded[i], now: now} : null);
        updates.push(upd);
    }
    if (updates.length > 0) {
        this._takeChecksum(native.membersChecksum);
        this.emit('updated', updates);
    }
    return updates;
};

Membership.prototype.shuffle = function shuffle() {  // _.shuffle (index.js:326-328)
    var a = this.members.slice();
    for (var i = a.length - 1; i > 0; i--) {
        var j = Math.floor(Math.random() * (i + 1));
        var t = a[i]; a[i] = a[j]; a[j] = t;
    }
    this.members = a;
};

Membership.prototype.startDampScoreDecayer = function startDampScoreDecayer() {  // index.js:330-350
    var self = this;
    if (this.decayTimer) { return; }
    schedule();
    function schedule() {
        if (!cfg(self.ringpop, 'dampScoringDecayEnabled', false)) { return; }
        self.decayTimer = self.setTimeout(function onTimeout() {
            self._decayMembersDampScore();
            schedule();
        }, cfg(self.ringpop, 'dampScoringDecayInterval', 1000));
        if (self.decayTimer && typeof self.decayTimer.unref === 'function') { self.decayTimer.unref(); }
    }
};

Membership.prototype.stopDampScoreDecayer = function stopDampScoreDecayer() {
    if (this.decayTimer) {
        this.clearTimeout(this.decayTimer);
        this.decayTimer = null;
    }
};

Membership.prototype.toString = function toString() {
    return JSON.stringify(this.members.map(function (m) { return m.address; }));
};

Membership.prototype._createMember = function _createMember(update) {  // index.js:364-374
    var self = this;
    var member = new Member(this.ringpop, update);
    member.on('suppressLimitExceeded', function onExceeded() { self.emit('memberSuppressLimitExceeded', member); });
    return member;
};

// _decayMembersDampScore (index.js:374-383): with device damp scoring one k_damp_decay sweep,
// then every Member takes its score and emits 'dampScoreDecayed' (new, old) as decayDampScore
// does (member.js:45-66).
Membership.prototype._decayMembersDampScore = function _decayMembersDampScore() {
    if (!this._damp()) {
        for (var i = 0; i < this.members.length; i++) { this.members[i].decayDampScore(); }
        return;
    }
    native.membersDampDecay(this._h, Date.now());
    var dump = native.membersDampDump(this._h);
    for (var j = 0; j < this.members.length; j++) {
        var m = this.members[j];
        var old = m.dampScore;
        m.dampScore = dump.score[this._ids[m.address]];
        if (old !== null && old !== undefined) { m.emit('dampScoreDecayed', m.dampScore, old); }
    }
};

Membership.prototype._updateMember = function _updateMember(update, isLocal) {  // index.js:386-397
    return this.update(update, isLocal);
};

Membership.prototype.destroy = function destroy() {
    this.stopDampScoreDecayer();
    native.destroy(this._h);
};

// initMembership(ringpop) — the export of lib/membership/index.js (399-418)
function initMembership(ringpop, options) {
    options = options || {};
    var membership = new Membership({ringpop: ringpop, device: options.device, capacity: options.capacity,
        setTimeout: options.setTimeout, clearTimeout: options.clearTimeout});
    membership.on('memberSuppressLimitExceeded', function () {});
    membership.startDampScoreDecayer();
    if (typeof ringpop.on === 'function') {
        ringpop.on('destroyed', function onDestroyed() { membership.stopDampScoreDecayer(); });
    }
    return membership;
}

// Seed the module cache so `require('<ringpopRoot>/lib/membership/index.js')` (the reference's
// index.js:51) returns initMembership. Call before requiring ringpop.
function install(ringpopRoot, options) {
    var file = path.join(ringpopRoot, 'lib', 'membership', 'index.js');
    var mod = new Module(file, null);
    mod.filename = file;
    mod.loaded = true;
    mod.exports = function (ringpop) { return initMembership(ringpop, options); };
    Module._cache[file] = mod;
    return mod.exports;
}

module.exports = initMembership;
module.exports.initMembership = initMembership;
module.exports.install = install;
module.exports.Membership = Membership;
module.exports.Member = Member;
module.exports.LocalMemberLeaveEvent = LocalMemberLeaveEvent;
