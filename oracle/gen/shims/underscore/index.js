// Stand-in for the absent npm `underscore` (^1.5.2, reference package.json:39), used ONLY to
// load the reference's lib/membership modules when generating golden vectors here.
// `_.defaults` is restated (the local-override path, lib/membership/member.js:76-81);
// every randomised helper (shuffle/sample/chain) throws: the golden harness injects its own
// deterministic schedule instead, so those must never be reached.
'use strict';
function defaults(obj) {
    for (var i = 1; i < arguments.length; i++) {
        var src = arguments[i];
        for (var k in src) {
            if (obj[k] === void 0) { obj[k] = src[k]; }
        }
    }
    return obj;
}
function unavailable(name) {
    return function () { throw new Error('underscore.' + name + ' is not available in the golden harness'); };
}
module.exports = {
    defaults: defaults,
    shuffle: unavailable('shuffle'),
    sample: unavailable('sample'),
    chain: unavailable('chain'),
    pluck: unavailable('pluck'),
};
