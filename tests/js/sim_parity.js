// sim_parity.js — runs the golden gossip cases (tests/golden/sim_golden.json: the reference
// modules driven through the round model) through the N-API GossipSim of ringpop-node_amd/js
// and compares every live node's checksum after every round. in.json (from
// tests/test_js_gpu.py) adds each case's names and inc0. Prints one JSON line.
'use strict';
var fs = require('fs');
var path = require('path');
var amd = require(path.join(__dirname, '..', '..', 'ringpop-node_amd', 'js'));

var input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
var fails = [], checks = 0;
input.cases.forEach(function (c) {
    var sim = new amd.GossipSim(c.names, {inc0: c.inc0, dead: c.dead, seed: c.seed,
        suspicionRounds: c.suspRounds, now0: c.now0, events: c.events || []});
    c.checksums.forEach(function (want, r) {
        sim.step(1);
        var got = Array.from(sim.checksums());
        checks++;
        if (JSON.stringify(got) !== JSON.stringify(want)) { fails.push(c.name + ' round ' + r); }
    });
    checks++;
    if (sim.round() !== c.checksums.length) { fails.push(c.name + ' round counter ' + sim.round()); }
    sim.destroy();
});
process.stdout.write(JSON.stringify({checks: checks, fails: fails.slice(0, 20), nfail: fails.length}) + '\n');
