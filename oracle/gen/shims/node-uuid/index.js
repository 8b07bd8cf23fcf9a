// Stand-in for the absent npm `node-uuid` (^1.4.3): Update ids (lib/membership/update.js:30)
// never affect membership state or checksums; a counter keeps them unique.
'use strict';
var n = 0;
module.exports = { v4: function v4() { n += 1; return 'golden-' + n; } };
