// wire_parity.js — the gossip wire bodies through the N-API addon (rpamd.node wireEncode /
// wireDecode -> rp_wire_encode / rp_wire_decode): every body of tests/golden/wire_golden.json
// (what the reference's Dissemination + protocol handlers wrote) encoded byte for byte, then
// decoded back. Prints one JSON line.
'use strict';
var fs = require('fs');
var path = require('path');
var amd = require(path.join(__dirname, '..', '..', 'ringpop-node_amd', 'js'));
var native = amd.native;

var input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
var ST = {alive: 0, suspect: 1, faulty: 2, leave: 3};
var BODY = {array: 0, ping: 1, pingResponse: 2, pingReq: 3, pingReqResponse: 4, joinResponse: 5};
var NULL = 0xFFFFFFFF;
var fails = [], checks = 0;
function eq(what, got, want) {
    checks++;
    if (JSON.stringify(got) !== JSON.stringify(want)) {
        fails.push({what: what, got: JSON.stringify(got).slice(0, 300), want: JSON.stringify(want).slice(0, 300)});
    }
}

var mm = new amd.MembershipMerge('0.0.0.0:0');
var h = mm._h;
function id(a) { return a === null || a === undefined ? NULL : native.membersIntern(h, [a])[0]; }

input.cases.forEach(function (c) {
    var recs = function (rows) {
        var n = rows.length, r = {addr: new Uint32Array(n), src: new Uint32Array(n), status: new Uint8Array(n),
            inc: new Float64Array(n), srcInc: new Float64Array(n), ids: new Uint8Array(36 * n)};
        rows.forEach(function (x, i) {
            r.addr[i] = id(x[0]); r.src[i] = id(x[3]); r.status[i] = ST[x[1]]; r.inc[i] = x[2];
            r.srcInc[i] = x[4] === null || x[4] === undefined ? NaN : x[4];
            if (x[5]) { for (var b = 0; b < 36; b++) { r.ids[36 * i + b] = x[5].charCodeAt(b); } }
        });
        return r;
    };
    var issue = recs(c.changes);
    var full = recs(c.members.map(function (m) { return [m[0], m[1], m[2], c.whoami, null, null]; }));
    var hdr = {checksum: Uint32Array.of(c.checksum), source: Uint32Array.of(id(c.whoami)),
        sourceInc: Float64Array.of(c.whoamiInc), target: Uint32Array.of(id(c.target)),
        pingStatus: Uint8Array.of(c.pingStatus ? 1 : 0), app: c.app};
    function enc(r, form, body) {
        var n = r.addr.length;
        var e = native.wireEncode(h, Uint32Array.of(0, n), r, form, BODY[body], hdr);
        return Buffer.from(e.bytes.buffer, 0, e.off[1]).toString();
    }
    eq(c.name + ' issueAs', enc(issue, 0, 'array'), c.out.issueAs);
    eq(c.name + ' ping', enc(issue, 0, 'ping'), c.out.ping);
    eq(c.name + ' pingResponse', enc(issue, 0, 'pingResponse'), c.out.pingResponse);
    eq(c.name + ' pingReq', enc(issue, 0, 'pingReq'), c.out.pingReq);
    eq(c.name + ' fullSync', enc(full, 1, 'array'), c.out.fullSync);
    eq(c.name + ' joinResponse', enc(full, 1, 'joinResponse'), c.out.joinResponse);
    // decode the reference's bodies back
    var kinds = ['ping', 'pingReq', 'pingReqResponse', 'joinResponse'];
    var texts = kinds.map(function (k) { return Buffer.from(c.out[k]); });
    var off = new Float64Array(texts.length + 1);
    texts.forEach(function (t, i) { off[i + 1] = off[i] + t.length; });
    var d = native.wireDecode(h, new Uint8Array(Buffer.concat(texts)), off, 4096);
    eq(c.name + ' decode err', Array.from(d.err), [0, 0, 0, 0]);
    eq(c.name + ' decode counts', d.recOff[1] - d.recOff[0], c.changes.length);
    eq(c.name + ' join count', d.recOff[4] - d.recOff[3], c.members.length);
    eq(c.name + ' pingReq target', d.target[1], id(c.target));
    eq(c.name + ' pingReq status', [d.pingStatus[1], d.pingStatus[2]], [0xFF, c.pingStatus ? 1 : 0]);
    eq(c.name + ' join coordinator / checksum', [d.source[3], d.checksum[3]], [id(c.whoami), c.checksum]);
    for (var i = 0; i < c.changes.length; i++) {
        var ch = c.changes[i];
        eq(c.name + ' rec ' + i, [d.addr[i], d.src[i], d.status[i], d.inc[i], isNaN(d.srcInc[i]) ? null : d.srcInc[i]],
            [id(ch[0]), id(ch[3]), ST[ch[1]], ch[2], ch[4]]);
    }
});
mm.destroy();
console.log(JSON.stringify({nfail: fails.length, checks: checks, fails: fails.slice(0, 20)}));
