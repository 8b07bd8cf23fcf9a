// index.js — the reference's JS API over the MI355X engine (rpamd.node -> librpamd.so).
//
// HashRing is a drop-in for ringpop's lib/ring/index.js (options.Ring plug point,
// reference index.js:107,133): same constructor options, methods, `checksum` property and
// events. The RB-tree is replaced by the sorted token table in HBM. Every hash, insert,
// remove, checksum and lookup runs in HIP kernels; with no device the constructor throws.
// Batched forms (lookupBatch / lookupNBatch / lookupNHashes) are the point of the engine:
// one kernel launch for a whole batch of keys.
//
// MembershipMerge is the device-side hot loop of Membership.update
// (lib/membership/index.js:249-324, member.js:71-202) and computeChecksum (48-75).
// GossipSim runs N full ringpop nodes in the deterministic round model (DESIGN.md §5).
'use strict';
var EventEmitter = require('events').EventEmitter;
var util = require('util');
var path = require('path');

var native;
try {
    native = require(path.join(__dirname, 'rpamd.node'));
} catch (e) {
    throw new Error('ringpop_amd: rpamd.node is not built (make -C ringpop-node_amd/js): ' + e.message);
}

var STATUS = ['alive', 'suspect', 'faulty', 'leave'];
var STATUS_CODE = {alive: 0, suspect: 1, faulty: 2, leave: 3};

function requireDevice(device) {
    var n = native.deviceCount();
    if (n <= device) {
        throw new Error('ringpop_amd: no HIP device ' + device + ' (visible: ' + n + ')');
    }
}

// new HashRing({replicaPoints, hashFunc, device}) — lib/ring/index.js:25-34.
function HashRing(options) {
    EventEmitter.call(this);
    this.options = options || {};
    this.replicaPoints = this.options.replicaPoints || 100;
    // options.hashFunc (index.js:29): a caller hash is evaluated here, in JS, and its values
    // are handed to the device as tokens / key hashes; the default is the device farmhash32.
    this.hashFunc = this.options.hashFunc || native.hash32;
    this._customHash = typeof this.options.hashFunc === 'function';
    this.device = this.options.device || 0;
    requireDevice(this.device);
    this._h = native.ringCreate(this.replicaPoints, this.device);
    // options.serviceIdleMs: single-key lookup / lookupN calls go through the resident lookup
    // service (rp_ring_service: a pinned request line polled by one device wave, no launch per
    // call; ~3.7 us against ~14 us with a launch). Default 20 ms of idle before the wave exits
    // (round 5: lookup is the per-request call of handleOrProxy); 0 turns it off.
    this.serviceIdleMs = this.options.serviceIdleMs === undefined ? 20 : this.options.serviceIdleMs >>> 0;
    if (this.serviceIdleMs) { native.ringService(this._h, this.serviceIdleMs); }
    // servers (index.js:32): name -> true in insertion order, as the reference keeps it (its
    // Object.keys order is getStats().servers). Host bookkeeping of the same add / remove
    // decisions the device makes; every change is checked against the device's answer.
    this.servers = {};
    this.checksum = null;
}
util.inherits(HashRing, EventEmitter);

HashRing.prototype.destroy = function destroy() {
    native.destroy(this._h);
};

HashRing.prototype._replicaTokens = function _replicaTokens(servers) {
    if (!this._customHash || !servers.length) { return null; }
    var R = this.replicaPoints;
    var t = new Uint32Array(servers.length * R);
    for (var j = 0; j < servers.length; j++) {
        for (var i = 0; i < R; i++) { t[j * R + i] = this.hashFunc(servers[j] + i) >>> 0; }
    }
    return t;
};

HashRing.prototype._refreshChecksum = function _refreshChecksum() {
    this.checksum = this._customHash ? this.hashFunc(native.ringChecksumString(this._h))
        : native.ringChecksum(this._h);
    this.emit('checksumComputed');
};

// The reference's decisions for a batch (index.js:60-94: adds in order, then removes in order,
// each tested with `!!this.servers[name]`), made before the device is touched: only the names
// that change go to the device, and the servers map is committed after the device succeeded, so
// the two never diverge (an add of a name the map already answers for, e.g. 'constructor', is
// skipped, as in the reference; see _applyPlan for removals of such names).
HashRing.prototype._planServers = function _planServers(add, remove) {
    var servers = this.servers, over = Object.create(null);
    function present(name) { return name in over ? over[name] : !!servers[name]; }
    var plan = {add: [], remove: []};
    for (var i = 0; i < add.length; i++) {
        if (!present(add[i])) { over[add[i]] = true; plan.add.push(add[i]); }
    }
    for (var j = 0; j < remove.length; j++) {
        if (present(remove[j])) { over[remove[j]] = false; plan.remove.push(remove[j]); }
    }
    return plan;
};

// A removal the reference accepts for a name the servers map only inherits ('constructor',
// 'toString', ...: `!!this.servers[name]` is true) deletes nothing and removes no token, yet
// still counts as a change (checksum recomputed, 'removed' emitted, ringChanged true). Such names
// never reach the device, which holds own names only (tests/golden/ring_ops_golden.json).
HashRing.prototype._applyPlan = function _applyPlan(plan) {
    var changed = plan.add.length + plan.remove.length > 0;
    if (!changed) { return false; }
    var own = Object.prototype.hasOwnProperty, servers = this.servers, adding = Object.create(null);
    for (var a = 0; a < plan.add.length; a++) { adding[plan.add[a]] = true; }
    // a name added earlier in this batch is on the device by the time its removal runs
    var remove = plan.remove.filter(function (n) { return own.call(servers, n) || n in adding; });
    if (plan.add.length + remove.length > 0) {
        var deviceChanged = native.ringAddRemove(this._h, plan.add, remove,
            this._replicaTokens(plan.add), this._replicaTokens(remove));
        if (!deviceChanged) {
            throw new Error('ringpop_amd: the device ring did not change for ' + JSON.stringify(plan));
        }
    }
    for (var i = 0; i < plan.add.length; i++) { servers[plan.add[i]] = true; }
    for (var j = 0; j < remove.length; j++) { delete servers[remove[j]]; }
    return true;
};

// addServer(name) — index.js:39-48
HashRing.prototype.addServer = function addServer(name) {
    if (this.hasServer(name)) { return; }
    this._applyPlan(this._planServers([name], []));
    this._refreshChecksum();
    this.emit('added', name);
};

// removeServer(name) — index.js:124-133
HashRing.prototype.removeServer = function removeServer(name) {
    if (!this.hasServer(name)) { return; }
    this._applyPlan(this._planServers([], [name]));
    this._refreshChecksum();
    this.emit('removed', name);
};

// addRemoveServers(add, remove) -> ringChanged — index.js:60-94 (no added/removed events,
// as in the reference).
HashRing.prototype.addRemoveServers = function addRemoveServers(serversToAdd, serversToRemove) {
    var changed = this._applyPlan(this._planServers(serversToAdd || [], serversToRemove || []));
    if (changed) { this._refreshChecksum(); }
    return changed;
};

// computeChecksum() — index.js:96-105 (the device recomputes it on every change; this
// re-reads it and emits, like the reference).
HashRing.prototype.computeChecksum = function computeChecksum() {
    this._refreshChecksum();
};

// getServerCount / getStats / hasServer — index.js:107-120, over the servers map as the
// reference reads them (no device round trip).
HashRing.prototype.getServerCount = function getServerCount() {
    return Object.keys(this.servers).length;
};

HashRing.prototype.getStats = function getStats() {
    return {checksum: this.checksum, servers: Object.keys(this.servers)};
};

HashRing.prototype.hasServer = function hasServer(name) {
    return !!this.servers[name];
};

// the device's own count / names (tests: coherence with the servers map)
HashRing.prototype.deviceServerCount = function deviceServerCount() {
    return native.ringServerCount(this._h);
};

// lookup(key) — index.js:145-154 (one key; use lookupBatch for throughput).
HashRing.prototype.lookup = function lookup(str) {
    if (this._customHash) { return this.lookupBatch([str])[0]; }
    return native.ringLookup1(this._h, str);
};

// lookupN(key, n) — index.js:157-189.
HashRing.prototype.lookupN = function lookupN(str, n) {
    if (this._customHash) { return this.lookupNBatch([str], n)[0]; }
    return native.ringLookupN1(this._h, str, n | 0);
};

HashRing.prototype._hashes = function _hashes(keys) {
    var h = new Uint32Array(keys.length);
    for (var i = 0; i < keys.length; i++) { h[i] = this.hashFunc(keys[i]) >>> 0; }
    return h;
};

HashRing.prototype._names = function _names(r, nrep) {
    var w = nrep > 1 ? nrep : 1;
    var out = new Array(r.counts.length);
    for (var i = 0; i < r.counts.length; i++) {
        var row = [];
        for (var j = 0; j < r.counts[i]; j++) { row.push(native.ringOwnerName(this._h, r.owners[i * w + j])); }
        out[i] = row;
    }
    return out;
};

// lookup() of every key, one launch.
HashRing.prototype.lookupBatch = function lookupBatch(keys) {
    if (this._customHash) {
        return this._names(native.ringLookupNHashes(this._h, this._hashes(keys), 1), 1)
            .map(function (row) { return row.length ? row[0] : null; });
    }
    return native.ringLookup(this._h, keys);
};

// lookupN(key, n) of every key, one launch.
HashRing.prototype.lookupNBatch = function lookupNBatch(keys, n) {
    if (this._customHash) {
        return this._names(native.ringLookupNHashes(this._h, this._hashes(keys), n), n);
    }
    return native.ringLookupN(this._h, keys, n);
};

// keysByDest of RingPop.handleOrProxyAll (index.js:609-667: _.groupBy(keys, this.lookup), :616)
// in one device pass: {dest: [keys in input order]}, dests in first-seen order (the order
// Object.keys(keysByDest) and RequestProxySend.lookupKeys, send.js:171-179, report). On an
// empty ring every key goes to whoami (RingPop.lookup, index.js:434-451).
HashRing.prototype.groupByOwner = function groupByOwner(keys, whoami) {
    var g = native.ringGroupKeys(this._h, this._customHash ? this._hashes(keys) : keys);
    var out = {};
    for (var d = 0; d < g.dests.length; d++) {
        var dest = g.dests[d] === null ? whoami : g.dests[d];
        var list = new Array(g.groupOff[d + 1] - g.groupOff[d]);
        for (var p = g.groupOff[d], j = 0; p < g.groupOff[d + 1]; p++, j++) { list[j] = keys[g.perm[p]]; }
        out[dest] = list;
    }
    return out;
};

// the name ringpop's handleOrProxyAll probes for (INTEGRATION.md): same function
HashRing.prototype.groupBy = HashRing.prototype.groupByOwner;

// RequestProxySend.lookupKeys (lib/request-proxy/send.js:171-179): distinct owners, first seen.
HashRing.prototype.lookupKeys = function lookupKeys(keys, whoami) {
    var g = native.ringGroupKeys(this._h, this._customHash ? this._hashes(keys) : keys);
    return g.dests.map(function (d) { return d === null ? whoami : d; });
};

// Id-level batch over precomputed key hashes: {owners: Uint32Array(ids, rows of max(n,1)),
// counts: Uint8Array}; ownerName(id) maps ids back to server names.
HashRing.prototype.lookupNHashes = function lookupNHashes(hashes, n) {
    return native.ringLookupNHashes(this._h, hashes, n);
};

HashRing.prototype.ownerName = function ownerName(id) {
    return native.ringOwnerName(this._h, id);
};

// MembershipMerge(whoami, {capacity, device}) — device state of one Membership: update()
// folds a changes array in order with the reference's override rules and returns the applied
// updates (Membership.update's return value, index.js:249-324); checksum as
// membership.checksum (null until the first applied update).
function MembershipMerge(whoami, options) {
    options = options || {};
    this.device = options.device || 0;
    requireDevice(this.device);
    this._h = native.membersCreate(options.capacity || 1024, this.device);
    this.whoami = whoami;
    native.membersSetLocal(this._h, native.membersIntern(this._h, [whoami])[0]);
}

MembershipMerge.prototype.destroy = function destroy() { native.destroy(this._h); };

MembershipMerge.prototype.update = function update(changes, nowMs) {
    changes = Array.isArray(changes) ? changes : [changes];
    var k = changes.length;
    var ids = native.membersIntern(this._h, changes.map(function (c) { return c.address; }));
    var st = new Uint8Array(k), inc = new Float64Array(k);
    for (var i = 0; i < k; i++) {
        var code = STATUS_CODE[changes[i].status];
        if (code === undefined) { throw new Error('ringpop_amd: unknown status ' + changes[i].status); }
        st[i] = code;
        inc[i] = changes[i].incarnationNumber;
    }
    var r = native.membersUpdate(this._h, ids, st, inc, nowMs === undefined ? Date.now() : nowMs);
    var applied = [];
    for (i = 0; i < k; i++) {
        if (!r.applied[i]) { continue; }
        var u = {};
        for (var key in changes[i]) { u[key] = changes[i][key]; }
        u.status = STATUS[r.status[i]];
        u.incarnationNumber = r.inc[i];
        applied.push(u);
    }
    return applied;
};

// set(stash) — Membership.set (index.js:208-247) over the changes stashed while !isReady
// (index.js:259-265; the caller keeps the stash and the Member objects): merged on the device
// (mergeMembershipChangesets, merge.js:22-51), set, checksum once. Returns the picked changes
// in first-seen order, the order new Member objects are appended in.
MembershipMerge.prototype.set = function set(stash) {
    var k = stash.length;
    var ids = native.membersIntern(this._h, stash.map(function (c) { return c.address; }));
    var st = new Uint8Array(k), inc = new Float64Array(k);
    for (var i = 0; i < k; i++) {
        var code = STATUS_CODE[stash[i].status];
        if (code === undefined) { throw new Error('ringpop_amd: unknown status ' + stash[i].status); }
        st[i] = code;
        inc[i] = stash[i].incarnationNumber;
    }
    var pick = native.membersSet(this._h, ids, st, inc);
    var out = [];
    for (i = 0; i < pick.length; i++) { out.push(stash[pick[i]]); }
    return out;
};

Object.defineProperty(MembershipMerge.prototype, 'checksum', {
    get: function () { return native.membersChecksum(this._h); }
});

MembershipMerge.prototype.computeChecksum = function computeChecksum() {
    return native.membersComputeChecksum(this._h);
};

MembershipMerge.prototype.generateChecksumString = function generateChecksumString() {
    return native.membersChecksumString(this._h);
};

// GossipSim(names, {inc0, dead, seed, suspicionRounds, now0, device})
function GossipSim(names, options) {
    options = options || {};
    this.n = names.length;
    this.device = options.device || 0;
    requireDevice(this.device);
    var inc0 = options.inc0 instanceof Float64Array ? options.inc0 : Float64Array.from(options.inc0);
    var dead = options.dead ? Uint8Array.from(options.dead) : new Uint8Array(this.n);
    // options.events: [[round, 'kill' | 'revive' | 'leave' | 'join', node], ...] (rp_sim_create_scenario)
    var kinds = {kill: 0, revive: 1, leave: 2, join: 3};
    var evs = options.events || [];
    var ev = new Uint32Array(3 * evs.length);
    evs.forEach(function (e, i) {
        ev[3 * i] = e[0];
        ev[3 * i + 1] = typeof e[1] === 'string' ? kinds[e[1]] : e[1];
        ev[3 * i + 2] = e[2];
    });
    this._h = native.simCreate(names, inc0, dead, options.seed || 0, options.suspicionRounds || 25,
        options.now0 || 0, this.device, ev);
}

GossipSim.prototype.destroy = function destroy() { native.destroy(this._h); };
GossipSim.prototype.step = function step(rounds) { native.simStep(this._h, rounds === undefined ? 1 : rounds); };
GossipSim.prototype.round = function round() { return native.simRound(this._h); };
GossipSim.prototype.checksums = function checksums() { return native.simChecksums(this._h, this.n); };
GossipSim.prototype.view = function view(v) { return native.simView(this._h, v, this.n); };
GossipSim.prototype.converged = function converged() { return native.simConverged(this._h); };
GossipSim.prototype.stats = function stats() { return native.simStats(this._h); };

module.exports = {
    HashRing: HashRing,
    MembershipMerge: MembershipMerge,
    GossipSim: GossipSim,
    hash32: native.hash32,
    native: native,
    STATUS: STATUS
};
