// ref_wire.js — runs the REFERENCE Dissemination (lib/gossip/dissemination.js from the
// reference checkout given on the command line) over recorded changes and records the JSON
// text ringpop would put on the wire. Golden-vector generator only (tests/golden/make_wire_golden.py).
//
//   node tests/golden/ref_wire.js <ref_root> <in.json> <out.json>
//
// Per case: recordChange() each change, then
//   issueAsSender()  -> JSON.stringify(changes)                     (dissemination.js:133-176)
//   fullSync()       -> JSON.stringify(changes)                     (dissemination.js:61-76)
//   the ping request body JSON.stringify({checksum, changes, source, sourceIncarnationNumber})
//   as ping-sender.js:71-76 builds it, and the ping response body {changes} of
//   server/protocol/ping.js:45-48 (issueAsReceiver from a sender no change came from);
//   the ping-req request {checksum, changes, source, sourceIncarnationNumber, target}
//   (ping-req-sender.js:75-81), the ping-req response {changes, pingStatus, target}
//   (server/protocol/ping-req.js:61-65) and the join response {app, coordinator, membership:
//   fullSync(), membershipChecksum} (server/protocol/join.js:128-133).
'use strict';
var fs = require('fs');
var path = require('path');
var EventEmitter = require('events').EventEmitter;
var util = require('util');

var refRoot = process.argv[2];
var input = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'));
var Dissemination = require(path.join(refRoot, 'lib/gossip/dissemination.js'));

function FakeRingpop(c) {
    EventEmitter.call(this);
    this.hostPort = c.whoami;
    this.logger = {debug: function () {}, info: function () {}, warn: function () {}, error: function () {}};
    this.ring = {getServerCount: function () { return c.serverCount; }};
    this.membership = {
        checksum: c.checksum,
        members: c.members.map(function (m) {
            return {address: m[0], status: m[1], incarnationNumber: m[2]};
        }),
        getIncarnationNumber: function () { return c.whoamiInc; }
    };
}
util.inherits(FakeRingpop, EventEmitter);
FakeRingpop.prototype.whoami = function () { return this.hostPort; };
FakeRingpop.prototype.stat = function () {};

var out = {cases: []};
input.cases.forEach(function (c) {
    var rp = new FakeRingpop(c);
    var d = new Dissemination(rp);
    rp.emit('ringChanged');  // maxPiggybackCount from the server count (dissemination.js:38-55)
    c.changes.forEach(function (ch) {
        var rec = {address: ch[0], status: ch[1], incarnationNumber: ch[2], source: ch[3],
                   sourceIncarnationNumber: ch[4]};
        if (ch[3] === null) { delete rec.source; }
        if (ch[4] === null) { delete rec.sourceIncarnationNumber; }
        if (ch[5] !== null) rec.id = ch[5];
        // Update field order (lib/membership/update.js:26-35); the wire order is _issueAs's
        d.recordChange(rec);
    });
    var sender = d.issueAsSender();
    var ping = JSON.stringify({
        checksum: rp.membership.checksum,
        changes: sender,
        source: rp.whoami(),
        sourceIncarnationNumber: rp.membership.getIncarnationNumber()
    });
    var resp = JSON.stringify({changes: d.issueAsReceiver('0.0.0.0:1', 1, rp.membership.checksum)});
    var pingReq = JSON.stringify({
        checksum: rp.membership.checksum,
        changes: sender,
        source: rp.whoami(),
        sourceIncarnationNumber: rp.membership.getIncarnationNumber(),
        target: c.target
    });
    var pingReqResp = JSON.stringify({
        changes: d.issueAsReceiver('0.0.0.0:1', 1, rp.membership.checksum),
        pingStatus: c.pingStatus,
        target: c.target
    });
    var join = JSON.stringify({
        app: c.app,
        coordinator: rp.whoami(),
        membership: d.fullSync(),
        membershipChecksum: rp.membership.checksum
    });
    out.cases.push({
        name: c.name,
        issueAs: JSON.stringify(sender),
        fullSync: JSON.stringify(d.fullSync()),
        ping: ping,
        pingResponse: resp,
        pingReq: pingReq,
        pingReqResponse: pingReqResp,
        joinResponse: join
    });
});
fs.writeFileSync(process.argv[4], JSON.stringify(out));
